"""The BASELINE.json configurations: XDP programs (hand-assembled eBPF) and synthetic packets.

SURVEY.md §8(d). Packet i of config c is a pure function of splitmix64(seed_c ^ i), so any shard
regenerates identical packets; seed_c = 0x6F62706C64000000 + c.

  C1  3-insn XDP_PASS (r0 = 2; r0 += 0; exit), 1k x 64 B, no maps
  C2  ~40-insn L2/L3 classifier, PASS for TCP/UDP/ICMP else DROP, per-proto ARRAY counters
  C3  5-tuple -> HASH lookup -> REDIRECT + hit counter, IMIX 64/576/1500 B, 64K flows preloaded
  C4  ~200-insn JEQ/JGT ACL (48 rules) on 1500 B packets, lane-divergence stress
  C5  C2-style parse + per-flow HASH counters {pkts, bytes}, 1M flows, 64 B packets, sharded
  C3-learn  C3 with flow learning: a miss inserts the flow (bpf_map_update_elem) — map-entry writes,
            order-dependent (the keyed path, xe_internal.h XE_MODE_SPEC / XE_MODE_CHAIN)
  C3-LRU    C3-learn over an LRU_HASH flow table (every lookup and update promotes; no eviction: the
            keyed path with the UsageList relinked by last touch)

All programs avoid JLT/JLE/JSET (rejected by emulator/inst.go Translate) and use only helper 1
(map lookup) — bpf_redirect does not exist in the reference emulator, so REDIRECT is `r0 = 4`.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from .asm import (Asm, JEQ, JGT, JNE, XDP_DROP, XDP_PASS, XDP_REDIRECT)
from .emulator import MAP_ARRAY, MAP_HASH, MAP_LRU_HASH, MapDef

SEED0 = 0x6F62706C64000000
M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = (x + np.uint64(0x9E3779B97F4A7C15)) & M64
        z = ((z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & M64
        z = ((z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & M64
        return z ^ (z >> np.uint64(31))


def rng_stream(config: int, idx: np.ndarray, k: int) -> np.ndarray:
    """k-th independent 64-bit random word for packets idx of config."""
    base = np.uint64(SEED0 + config) ^ idx.astype(np.uint64)
    return splitmix64(splitmix64(base) ^ np.uint64((k * 0xD1B54A32D192ED03) & 0xFFFFFFFFFFFFFFFF))


@dataclass
class Workload:
    name: str
    program: list[int]
    maps: list[tuple[MapDef, bytes | None]]
    map_entries: dict[int, tuple[np.ndarray, np.ndarray]] = field(default_factory=dict)  # idx -> (keys, vals)
    pkt_size: int | np.ndarray = 64
    description: str = ""


# ----------------------------------------------------------------------------- programs
def prog_c1() -> list[int]:
    a = Asm()
    a.mov64(0, XDP_PASS).add64(0, 0).exit()
    return a.assemble()


def _parse_eth(a: Asm, drop: str) -> None:
    """r6 = data, r7 = data_end, r3 = ethertype (LE-loaded), r4 = L3 offset; VLAN aware."""
    a.ldx(4, 6, 1, 0)          # r6 = ctx->data        (aliases the ctx object)
    a.ldx(4, 7, 1, 4)          # r7 = ctx->data_end
    a.mov64(2, src=6).add64(2, 14)
    a.jmp(JGT, 2, drop, src=7)             # if data + 14 > data_end: drop
    a.ldx(2, 3, 6, 12)                     # ethertype, read little endian
    a.mov64(4, 14)
    a.jmp(JNE, 3, "novlan", imm=0x0081)    # 0x8100 in network order
    a.mov64(2, src=6).add64(2, 18)
    a.jmp(JGT, 2, drop, src=7)
    a.ldx(2, 3, 6, 16)
    a.mov64(4, 18)
    a.label("novlan")


def prog_c2(rmw: bool = False) -> list[int]:
    """L2/L3 classifier: proto of IPv4/IPv6, count per proto in ARRAY map 1, PASS TCP/UDP/ICMP.
    rmw: the counter is bumped the way `value->packets++` compiles without __sync_fetch_and_add
    (load, add, store: an ordered read-modify-write unless lifted, xe_runtime.cpp lift_rmw)."""
    a = Asm()
    _parse_eth(a, "drop")
    a.jmp(JEQ, 3, "ipv4", imm=0x0008)      # 0x0800
    a.jmp(JEQ, 3, "ipv6", imm=0xDD86)      # 0x86dd
    a.ja("drop")
    a.label("ipv4")
    a.mov64(2, src=6).add64(2, src=4)      # r2 = data + l3off (pointer stays a MemoryPtr)
    a.mov64(5, src=2).add64(5, 20)
    a.jmp(JGT, 5, "drop", src=7)
    a.ldx(1, 8, 2, 9)                      # r8 = ip->protocol
    a.ja("count")
    a.label("ipv6")
    a.mov64(2, src=6).add64(2, src=4)
    a.mov64(5, src=2).add64(5, 40)
    a.jmp(JGT, 5, "drop", src=7)
    a.ldx(1, 8, 2, 6)                      # r8 = ip6->nexthdr
    a.label("count")
    a.stx(4, 10, -4, 8)                    # key = proto (u32 on the stack)
    a.ld_map(1, 1)
    a.mov64(2, src=10).add64(2, -4)
    a.call(1)                              # bpf_map_lookup_elem
    a.jmp(JEQ, 0, "verdict", imm=0)        # NULL (IMM 0) -> skip; a pointer never compares
    if rmw:
        a.ldx(8, 1, 0, 0).add64(1, 1).stx(8, 0, 0, 1)  # *(u64 *)(r0 + 0) += 1, not atomic
    else:
        a.mov64(1, 1)
        a.xadd(8, 0, 0, 1)                 # lock *(u64 *)(r0 + 0) += 1
    a.label("verdict")
    a.mov64(0, XDP_PASS)
    a.jmp(JEQ, 8, "out", imm=6)            # TCP
    a.jmp(JEQ, 8, "out", imm=17)           # UDP
    a.jmp(JEQ, 8, "out", imm=1)            # ICMP
    a.label("drop")
    a.mov64(0, XDP_DROP)
    a.label("out")
    a.exit()
    return a.assemble()


def _tuple_key(a: Asm, l3: str = "r6+14") -> None:
    """16-byte 5-tuple key on the stack at r10-16 from an IPv4 header at r2 (TCP/UDP ports)."""
    a.ldx(4, 3, 2, 12).stx(4, 10, -16, 3)   # saddr
    a.ldx(4, 3, 2, 16).stx(4, 10, -12, 3)   # daddr
    a.ldx(2, 3, 2, 20).stx(2, 10, -8, 3)    # sport
    a.ldx(2, 3, 2, 22).stx(2, 10, -6, 3)    # dport
    a.ldx(1, 3, 2, 9).stx(1, 10, -4, 3)     # proto
    a.st(1, 10, -3, 0)                      # pad[3] = 0
    a.st(2, 10, -2, 0)


def prog_c3() -> list[int]:
    """5-tuple -> HASH map 1 lookup; hit: hits += 1, REDIRECT (flow_id != 0); miss: PASS."""
    a = Asm()
    _parse_eth(a, "pass")
    a.jmp(JNE, 3, "pass", imm=0x0008)
    a.mov64(2, src=6).add64(2, src=4)
    a.mov64(5, src=2).add64(5, 24)
    a.jmp(JGT, 5, "pass", src=7)
    _tuple_key(a)
    a.ld_map(1, 1)
    a.mov64(2, src=10).add64(2, -16)
    a.call(1)
    a.jmp(JEQ, 0, "pass", imm=0)
    a.mov64(1, 1)
    a.xadd(8, 0, 8, 1)                      # value.hits += 1
    a.ldx(8, 3, 0, 0)                       # flow_id
    a.jmp(JEQ, 3, "pass", imm=0)
    a.mov64(0, XDP_REDIRECT)
    a.exit()
    a.label("pass")
    a.mov64(0, XDP_PASS)
    a.exit()
    return a.assemble()


def prog_c3learn() -> list[int]:
    """C3 with flow learning: hit -> hits += 1, REDIRECT; miss -> insert {flow_id = saddr | 1 << 32,
    hits = 1} (bpf_map_update_elem, BPF_ANY), PASS. Later packets of a learned flow hit it."""
    a = Asm()
    _parse_eth(a, "pass")
    a.jmp(JNE, 3, "pass", imm=0x0008)
    a.mov64(2, src=6).add64(2, src=4)
    a.mov64(5, src=2).add64(5, 24)
    a.jmp(JGT, 5, "pass", src=7)
    _tuple_key(a)
    a.ld_map(1, 1)
    a.mov64(2, src=10).add64(2, -16)
    a.call(1)
    a.jmp(JEQ, 0, "learn", imm=0)
    a.mov64(1, 1)
    a.xadd(8, 0, 8, 1)                      # value.hits += 1
    a.ldx(8, 3, 0, 0)                       # flow_id
    a.jmp(JEQ, 3, "pass", imm=0)
    a.mov64(0, XDP_REDIRECT)
    a.exit()
    a.label("learn")
    a.ldx(4, 3, 10, -16)                    # saddr from the key
    a.mov64(4, 1).alu64(0x60, 4, 32)        # r4 = 1 << 32 (LSH)
    a.alu64(0x40, 3, src=4)                 # flow_id = saddr | 1 << 32 (OR)
    a.stx(8, 10, -32, 3)
    a.st(8, 10, -24, 1)                     # hits = 1
    a.ld_map(1, 1)
    a.mov64(2, src=10).add64(2, -16)
    a.mov64(3, src=10).add64(3, -32)
    a.mov64(4, 0)                           # BPF_ANY
    a.call(2)                               # bpf_map_update_elem
    a.label("pass")
    a.mov64(0, XDP_PASS)
    a.exit()
    return a.assemble()


ACL_RULES = 48


def acl_rules() -> list[tuple[int, int, int, int]]:
    """(saddr_le, proto, dport_max_le, action) for each rule."""
    r = []
    idx = np.arange(ACL_RULES, dtype=np.uint64)
    w = rng_stream(4, idx + np.uint64(1 << 40), 7)
    for k in range(ACL_RULES):
        saddr = int(0x0A000000 | (k << 8) | 1)        # 10.0.k.1 (host order)
        saddr_le = int.from_bytes(saddr.to_bytes(4, "big"), "little")
        proto = 6 if k % 3 else 17
        dport_max = 1024 + int(w[k] % 30000)
        action = XDP_PASS if k % 2 == 0 else XDP_DROP
        r.append((saddr_le, proto, dport_max, action))
    return r


def prog_c4() -> list[int]:
    """Branchy ACL: first matching rule wins; default DROP. 4 instructions per rule."""
    a = Asm()
    _parse_eth(a, "deny")
    a.jmp(JNE, 3, "deny", imm=0x0008)
    a.mov64(2, src=6).add64(2, src=4)
    a.mov64(5, src=2).add64(5, 24)
    a.jmp(JGT, 5, "deny", src=7)
    a.ldx(4, 8, 2, 12)                      # saddr (LE)
    a.ldx(1, 9, 2, 9)                       # proto
    a.ldx(2, 5, 2, 22)                      # dport (LE u16)
    for k, (saddr, proto, dmax, action) in enumerate(acl_rules()):
        nxt = f"r{k + 1}"
        a.label(f"r{k}")
        a.jmp(JNE, 8, nxt, imm=saddr if saddr < 2**31 else saddr - 2**32, wide=False)
        a.jmp(JNE, 9, nxt, imm=proto)
        a.jmp(JGT, 5, nxt, imm=dmax)
        a.ja("allow" if action == XDP_PASS else "deny")
    a.label(f"r{ACL_RULES}")
    a.label("deny")
    a.mov64(0, XDP_DROP)
    a.exit()
    a.label("allow")
    a.mov64(0, XDP_PASS)
    a.exit()
    return a.assemble()


def prog_c5() -> list[int]:
    """C2-style parse + per-flow HASH counters {pkts, bytes}; verdict PASS (DROP if not IPv4)."""
    a = Asm()
    _parse_eth(a, "drop")
    a.jmp(JNE, 3, "drop", imm=0x0008)
    a.mov64(2, src=6).add64(2, src=4)
    a.mov64(5, src=2).add64(5, 24)
    a.jmp(JGT, 5, "drop", src=7)
    _tuple_key(a)
    a.ld_map(1, 1)
    a.mov64(2, src=10).add64(2, -16)
    a.call(1)
    a.jmp(JEQ, 0, "pass", imm=0)
    a.mov64(1, 1)
    a.xadd(8, 0, 0, 1)                      # pkts += 1
    a.mov64(1, src=7).sub64(1, src=6)       # len = data_end - data (stays a MemoryPtr; value = len)
    a.xadd(8, 0, 8, 1)                      # bytes += len
    a.label("pass")
    a.mov64(0, XDP_PASS)
    a.exit()
    a.label("drop")
    a.mov64(0, XDP_DROP)
    a.exit()
    return a.assemble()


def prog_bpf2bpf() -> list[int]:
    """Call-heavy analogue of the reference's cmd/examples/bpf_to_bpf/src/xdp.c: the XDP section parses
    Ethernet / IPv4 and calls a non-inlined sub-program (bpf-to-bpf, emulator/inst_call_bpf.go:18-44)
    once for the IP protocol's stats and once more for the TCP or UDP destination port's stats. The
    sub-program looks the key up and either bumps {pkts, bytes} with plain loads / stores (the C
    `stats_ptr->pkts++`, lifted to adds) or inserts a fresh {1, framesize} (bpf_map_update_elem).
    HASH maps instead of the example's LRU_PERCPU_HASH (the same helper calls). Maps: 1 protocols,
    2 TCP ports, 3 UDP ports (4-byte keys, {u64 pkts, u64 bytes})."""
    a = Asm()
    a.ldx(4, 6, 1, 0).ldx(4, 7, 1, 4)
    a.mov64(2, src=6).add64(2, 14)
    a.jmp(JGT, 2, "pass", src=7)
    a.ldx(2, 3, 6, 12)
    a.jmp(JNE, 3, "pass", imm=0x0008)
    a.mov64(9, src=6).add64(9, 14)
    a.mov64(5, src=9).add64(5, 24)
    a.jmp(JGT, 5, "pass", src=7)
    a.ldx(2, 8, 9, 2).end(8, 16, to_be=False)  # framesize = ntohs(ip->tot_len) (to_le swaps, A10)
    a.ld_map(1, 1).ldx(1, 2, 9, 9).mov64(3, src=8)
    a.call_bpf("inc")                          # inc_ip_proto(proto, framesize)
    a.ldx(1, 2, 9, 9)
    a.jmp(JEQ, 2, "tcp", imm=6)
    a.jmp(JNE, 2, "pass", imm=17)
    a.ld_map(1, 3).ja("port")
    a.label("tcp").ld_map(1, 2)
    a.label("port").ldx(2, 2, 9, 22).end(2, 16, to_be=False)  # le_dest = ntohs(dest)
    a.mov64(3, src=8)
    a.call_bpf("inc")                          # inc_tcp / inc_udp(dest, framesize)
    a.label("pass").mov64(0, XDP_PASS).exit()
    # inc(map r1, key r2, framesize r3): lookup; hit: pkts++, bytes += framesize; miss: insert {1, size}
    a.label("inc")
    a.mov64(6, src=1).mov64(7, src=3)
    a.stx(4, 10, -8, 2)
    a.mov64(2, src=10).add64(2, -8).call(1)
    a.jmp(JEQ, 0, "new", imm=0)
    a.ldx(8, 1, 0, 0).add64(1, 1).stx(8, 0, 0, 1)
    a.ldx(8, 1, 0, 8).add64(1, src=7).stx(8, 0, 8, 1)
    a.mov64(0, 0).exit()
    a.label("new")
    a.st(8, 10, -24, 1).stx(8, 10, -16, 7)
    a.mov64(1, src=6).mov64(2, src=10).add64(2, -8).mov64(3, src=10).add64(3, -24).mov64(4, 0).call(2)
    a.mov64(0, 0).exit()
    return a.assemble()


BPF2BPF_PORTS = 1 << 14   # the C5 stream's destination ports (flow_tuples: 14 bits)


def bpf2bpf_map_entries() -> list[tuple[np.ndarray, np.ndarray]]:
    """Every key the stream uses preloaded (protocols 0..255, ports 0..16383): no inserts, so the batch
    stays commutative (lifted adds)."""
    protos = np.arange(256, dtype=np.uint32).view(np.uint8).reshape(-1, 4)
    ports = np.arange(BPF2BPF_PORTS, dtype=np.uint32).view(np.uint8).reshape(-1, 4)
    return [(protos, np.zeros((256, 16), np.uint8)), (ports, np.zeros((BPF2BPF_PORTS, 16), np.uint8)),
            (ports.copy(), np.zeros((BPF2BPF_PORTS, 16), np.uint8))]


# ----------------------------------------------------------------------------- packets
ETH_IPV4 = 0x0800
ETH_IPV6 = 0x86DD
ETH_ARP = 0x0806


def _be16(arr: np.ndarray, col: int, v: np.ndarray) -> None:
    arr[:, col] = (v >> 8) & 0xFF
    arr[:, col + 1] = v & 0xFF


def _be32(arr: np.ndarray, col: int, v: np.ndarray) -> None:
    for b in range(4):
        arr[:, col + b] = (v >> (8 * (3 - b))) & 0xFF


def headers_c2(idx: np.ndarray, hdr: int = 64) -> np.ndarray:
    """First `hdr` bytes of C2 packets: 60% v4/TCP, 25% v4/UDP, 5% v4/ICMP, 5% v6/TCP, 5% ARP; 3% VLAN."""
    n = len(idx)
    h = np.zeros((n, hdr), dtype=np.uint8)
    r0 = rng_stream(2, idx, 0)
    r1 = rng_stream(2, idx, 1)
    # random MACs / payload noise
    for b in range(12):
        h[:, b] = (r1 >> np.uint64(8 * (b % 8))) & np.uint64(0xFF)
    mix = (r0 % np.uint64(100)).astype(np.int64)
    vlan = ((r0 >> np.uint64(20)) % np.uint64(100)).astype(np.int64) < 3
    kind = np.select([mix < 60, mix < 85, mix < 90, mix < 95], [0, 1, 2, 3], 4)
    l3 = np.where(vlan, 18, 14)
    et = np.select([kind <= 2, kind == 3], [ETH_IPV4, ETH_IPV6], ETH_ARP).astype(np.int64)
    rows_v = np.nonzero(vlan)[0]
    rows_n = np.nonzero(~vlan)[0]
    h[rows_v, 12], h[rows_v, 13] = 0x81, 0x00
    h[rows_v, 14] = ((r1[rows_v] >> np.uint64(40)) & np.uint64(0x0F)).astype(np.uint8)
    h[rows_v, 15] = 0x64
    h[rows_v, 16] = (et[rows_v] >> 8) & 0xFF
    h[rows_v, 17] = et[rows_v] & 0xFF
    h[rows_n, 12] = (et[rows_n] >> 8) & 0xFF
    h[rows_n, 13] = et[rows_n] & 0xFF
    proto = np.select([kind == 0, kind == 1, kind == 2, kind == 3], [6, 17, 1, 6], 0).astype(np.uint8)
    for off in (14, 18):
        rows = np.nonzero((l3 == off) & (kind <= 2))[0]
        h[rows, off] = 0x45
        h[rows, off + 8] = 64
        h[rows, off + 9] = proto[rows]
        rows6 = np.nonzero((l3 == off) & (kind == 3))[0]
        h[rows6, off] = 0x60
        h[rows6, off + 6] = proto[rows6]
        h[rows6, off + 7] = 64
    return h


def flow_tuples(config: int, fid: np.ndarray) -> np.ndarray:
    """(saddr_be, daddr_be, sport_be, dport_be, proto) as a (n, 13) byte array for flow ids."""
    w = rng_stream(config, fid.astype(np.uint64) + np.uint64(1 << 48), 11)
    w2 = rng_stream(config, fid.astype(np.uint64) + np.uint64(1 << 48), 12)
    t = np.zeros((len(fid), 13), dtype=np.uint8)
    saddr = (np.uint64(0x0A000000) | (w & np.uint64(0xFFFFFF))).astype(np.int64)
    daddr = (np.uint64(0xC0A80000) | ((w >> np.uint64(24)) & np.uint64(0xFFFF))).astype(np.int64)
    sport = ((w2 & np.uint64(0xFFFF)) | np.uint64(1024)).astype(np.int64) & 0xFFFF
    dport = ((w2 >> np.uint64(16)) & np.uint64(0x3FFF)).astype(np.int64)
    proto = np.where((w2 >> np.uint64(40)) & np.uint64(1), 6, 17)
    _be32(t, 0, saddr)
    _be32(t, 4, daddr)
    _be16(t, 8, sport)
    _be16(t, 10, dport)
    t[:, 12] = proto
    return t


def key_from_tuple(t: np.ndarray) -> np.ndarray:
    """16-byte map key exactly as the programs build it on the stack (fields kept in packet order)."""
    k = np.zeros((len(t), 16), dtype=np.uint8)
    k[:, 0:4] = t[:, 0:4]
    k[:, 4:8] = t[:, 4:8]
    k[:, 8:10] = t[:, 8:10]
    k[:, 10:12] = t[:, 10:12]
    k[:, 12] = t[:, 12]
    return k


def _ipv4_l4_headers(config: int, idx: np.ndarray, tup: np.ndarray, hdr: int = 64) -> np.ndarray:
    n = len(idx)
    h = np.zeros((n, hdr), dtype=np.uint8)
    r1 = rng_stream(config, idx, 1)
    for b in range(12):
        h[:, b] = (r1 >> np.uint64(8 * (b % 8))) & np.uint64(0xFF)
    h[:, 12], h[:, 13] = 0x08, 0x00
    h[:, 14] = 0x45
    h[:, 22] = 64
    h[:, 23] = tup[:, 12]
    h[:, 26:30] = tup[:, 0:4]
    h[:, 30:34] = tup[:, 4:8]
    h[:, 34:36] = tup[:, 8:10]
    h[:, 36:38] = tup[:, 10:12]
    return h


C3_FLOWS = 65536
C3_MAX = 1 << 20
C5_FLOWS = 1 << 20
C5_MAX = 1 << 20
C3_NEW_FLOWS = 1 << 18   # C3-learn: the flows misses come from (learned on first sight)


def zipf_ranks(u: np.ndarray, nflows: int, s: float = 1.1) -> np.ndarray:
    """Inverse-CDF Zipf(s) sample over ranks 0..nflows-1 from uniform u in [0,1)."""
    w = 1.0 / np.power(np.arange(1, nflows + 1, dtype=np.float64), s)
    cdf = np.cumsum(w)
    cdf /= cdf[-1]
    return np.minimum(np.searchsorted(cdf, u, side="right"), nflows - 1)


def headers_c3(idx: np.ndarray, hdr: int = 64) -> np.ndarray:
    r0 = rng_stream(3, idx, 0)
    u = (r0 >> np.uint64(11)).astype(np.float64) / float(1 << 53)
    hit = (rng_stream(3, idx, 2) % np.uint64(10)) != 0          # 90% hits
    fid = zipf_ranks(u, C3_FLOWS).astype(np.uint64)
    miss_id = np.uint64(C3_FLOWS) + (rng_stream(3, idx, 3) % np.uint64(1 << 30))
    fid = np.where(hit, fid, miss_id)
    return _ipv4_l4_headers(3, idx, flow_tuples(3, fid), hdr)


def headers_c3learn(idx: np.ndarray, hdr: int = 64) -> np.ndarray:
    """C3's stream, its 10% misses drawn from C3_NEW_FLOWS flows that are not preloaded."""
    r0 = rng_stream(3, idx, 0)
    u = (r0 >> np.uint64(11)).astype(np.float64) / float(1 << 53)
    hit = (rng_stream(3, idx, 2) % np.uint64(10)) != 0
    fid = zipf_ranks(u, C3_FLOWS).astype(np.uint64)
    new_id = np.uint64(C3_FLOWS) + (rng_stream(3, idx, 3) % np.uint64(C3_NEW_FLOWS))
    fid = np.where(hit, fid, new_id)
    return _ipv4_l4_headers(3, idx, flow_tuples(3, fid), hdr)


C3LRU_COLD_BASE = 1 << 21   # C3-LRU-full: flow ids of the stale entries that fill the table
C3LRU_NEW_BASE = 1 << 22    # ... and of the flows its misses learn (disjoint from every preloaded one)


def headers_c3lrufull(idx: np.ndarray, hdr: int = 64) -> np.ndarray:
    """C3-learn's stream for the full LRU table: hits Zipf over the 64K hot flows, the 10% misses drawn
    from C3_NEW_FLOWS flows that are in the table at no point before they are learned."""
    r0 = rng_stream(3, idx, 0)
    u = (r0 >> np.uint64(11)).astype(np.float64) / float(1 << 53)
    hit = (rng_stream(3, idx, 2) % np.uint64(10)) != 0
    fid = zipf_ranks(u, C3_FLOWS).astype(np.uint64)
    new_id = np.uint64(C3LRU_NEW_BASE) + (rng_stream(3, idx, 3) % np.uint64(C3_NEW_FLOWS))
    fid = np.where(hit, fid, new_id)
    return _ipv4_l4_headers(3, idx, flow_tuples(3, fid), hdr)


def c3lrufull_map_entries() -> tuple[np.ndarray, np.ndarray]:
    """A full flow table (C3_MAX entries) in UsageList order of insertion: first the stale flows nobody
    sends any more (C3_MAX - 64K of them), then the 64K hot flows from the coldest to the hottest, so the
    hottest flow (rank 0) is the most recently used — the order steady traffic leaves an LRU table in."""
    cold = np.uint64(C3LRU_COLD_BASE) + np.arange(C3_MAX - C3_FLOWS, dtype=np.uint64)
    hot = np.arange(C3_FLOWS - 1, -1, -1, dtype=np.int64).astype(np.uint64)
    fid = np.concatenate([cold, hot])
    keys = key_from_tuple(flow_tuples(3, fid))
    vals = np.zeros((len(fid), 16), dtype=np.uint8)
    vals[:, 0:8] = (fid + np.uint64(1)).view(np.uint8).reshape(-1, 8)
    return keys, vals


def sizes_c3(idx: np.ndarray) -> np.ndarray:
    """IMIX-like {64: 7, 576: 4, 1500: 1}."""
    m = (rng_stream(3, idx, 5) % np.uint64(12)).astype(np.int64)
    return np.where(m < 7, 64, np.where(m < 11, 576, 1500)).astype(np.int64)


def headers_c4(idx: np.ndarray, hdr: int = 64) -> np.ndarray:
    rules = acl_rules()
    r0 = rng_stream(4, idx, 0)
    tgt = (r0 % np.uint64(ACL_RULES + 1)).astype(np.int64)      # hit position uniform over 0..48
    w = rng_stream(4, idx, 1)
    t = np.zeros((len(idx), 13), dtype=np.uint8)
    saddr = (np.uint64(0x0B000000) | (w & np.uint64(0xFFFFFF))).astype(np.int64)   # 11.x.x.x: no rule
    proto = np.where(w >> np.uint64(60) & np.uint64(1), 6, 17).astype(np.int64)
    dport = ((w >> np.uint64(32)) & np.uint64(0xFFFF)).astype(np.int64)
    for k, (s_le, p, dmax, _) in enumerate(rules):
        rows = tgt == k
        saddr[rows] = int.from_bytes(int(s_le).to_bytes(4, "little"), "big")
        proto[rows] = p
        dport_le = (w[rows] >> np.uint64(8)).astype(np.int64) % (dmax + 1)   # LE value <= dmax
        dport[rows] = ((dport_le & 0xFF) << 8) | ((dport_le >> 8) & 0xFF)     # stored big endian
    _be32(t, 0, saddr)
    _be32(t, 4, np.full(len(idx), 0xC0A80001, dtype=np.int64))
    _be16(t, 8, np.full(len(idx), 40000, dtype=np.int64))
    _be16(t, 10, dport)
    t[:, 12] = proto
    return _ipv4_l4_headers(4, idx, t, hdr)


def headers_c5(idx: np.ndarray, hdr: int = 64) -> np.ndarray:
    fid = (rng_stream(5, idx, 0) % np.uint64(C5_FLOWS + C5_FLOWS // 16))   # ~6% misses
    return _ipv4_l4_headers(5, idx, flow_tuples(5, fid), hdr)


def headers_bpf2bpf(idx: np.ndarray, hdr: int = 64) -> np.ndarray:
    """C5's stream with the IPv4 total length filled in (64-byte frames: 50), the framesize the
    call-heavy program accounts."""
    h = headers_c5(idx, hdr)
    h[:, 16], h[:, 17] = 0, 50
    return h


def c3_map_entries() -> tuple[np.ndarray, np.ndarray]:
    fid = np.arange(C3_FLOWS, dtype=np.uint64)
    keys = key_from_tuple(flow_tuples(3, fid))
    vals = np.zeros((C3_FLOWS, 16), dtype=np.uint8)
    vals[:, 0:8] = (fid + np.uint64(1)).view(np.uint8).reshape(-1, 8)   # flow_id = fid + 1 (LE)
    return keys, vals


def c5_map_entries() -> tuple[np.ndarray, np.ndarray]:
    fid = np.arange(C5_FLOWS, dtype=np.uint64)
    keys = key_from_tuple(flow_tuples(5, fid))
    return keys, np.zeros((C5_FLOWS, 16), dtype=np.uint8)


CONFIGS = {
    "c1": dict(program=prog_c1, pkt=64, n=1024),
    "c2": dict(program=prog_c2, pkt=64, n=16 * 1024 * 1024),
    "c2rmw": dict(program=lambda: prog_c2(rmw=True), pkt=64, n=16 * 1024 * 1024),
    "c3": dict(program=prog_c3, pkt="imix", n=16 * 1024 * 1024),
    "c3learn": dict(program=prog_c3learn, pkt="imix", n=16 * 1024 * 1024),
    "c3lru": dict(program=prog_c3learn, pkt="imix", n=16 * 1024 * 1024),
    "c3lrufull": dict(program=prog_c3learn, pkt="imix", n=16 * 1024 * 1024),
    "c4": dict(program=prog_c4, pkt=1500, n=16 * 1024 * 1024),
    # C4 in AF_XDP frames: 2-KiB chunks, the packet after the 256-byte XDP headroom (xsk.go:695-701
    # descriptors into a UMEM of fixed-size frames) instead of back to back
    "c4f": dict(program=prog_c4, pkt=1500, n=16 * 1024 * 1024, frame=(2048, 256)),
    "c5": dict(program=prog_c5, pkt=64, n=256 * 1024 * 1024),
    "bpf2bpf": dict(program=prog_bpf2bpf, pkt=64, n=4 * 1024 * 1024),
}


def workload_maps(name: str) -> list[tuple[MapDef, tuple[np.ndarray, np.ndarray] | None]]:
    if name in ("c2", "c2rmw"):
        return [(MapDef(MAP_ARRAY, 4, 8, 256), None)]
    if name in ("c3", "c3learn"):
        return [(MapDef(MAP_HASH, 16, 16, C3_MAX), c3_map_entries())]
    if name == "c3lru":  # the learning flow table as an LRU_HASH (room for every flow: no eviction)
        return [(MapDef(MAP_LRU_HASH, 16, 16, C3_MAX), c3_map_entries())]
    if name == "c3lrufull":  # the LRU flow table full: every learned flow evicts the least recently used
        return [(MapDef(MAP_LRU_HASH, 16, 16, C3_MAX), c3lrufull_map_entries())]
    if name == "c5":
        return [(MapDef(MAP_HASH, 16, 16, C5_MAX), c5_map_entries())]
    if name == "bpf2bpf":
        e = bpf2bpf_map_entries()
        return [(MapDef(MAP_HASH, 4, 16, 256), e[0]), (MapDef(MAP_HASH, 4, 16, BPF2BPF_PORTS), e[1]),
                (MapDef(MAP_HASH, 4, 16, BPF2BPF_PORTS), e[2])]
    return []


def headers(name: str, idx: np.ndarray, hdr: int = 64) -> np.ndarray:
    if name in ("c1",):
        h = np.zeros((len(idx), hdr), dtype=np.uint8)
        r = rng_stream(1, idx, 0)
        for b in range(hdr):
            h[:, b] = (r >> np.uint64(8 * (b % 8))) & np.uint64(0xFF)
        return h
    return {"c2": headers_c2, "c2rmw": headers_c2, "c3": headers_c3, "c3learn": headers_c3learn, "c3lru": headers_c3learn, "c3lrufull": headers_c3lrufull, "c4": headers_c4, "c4f": headers_c4,
            "c5": headers_c5, "bpf2bpf": headers_bpf2bpf}[name](idx, hdr)


def packet_sizes(name: str, idx: np.ndarray) -> np.ndarray:
    p = CONFIGS[name]["pkt"]
    if p == "imix":
        return sizes_c3(idx)
    return np.full(len(idx), int(p), dtype=np.int64)


def packet_offsets(name: str, sizes: np.ndarray) -> tuple[np.ndarray, int]:
    """UMEM address of every packet and the UMEM size: back to back (a compacted UMEM / pcap-style buffer),
    or one fixed-size frame per packet after a headroom (configs with `frame`: an AF_XDP UMEM)."""
    n = len(sizes)
    frame = CONFIGS.get(name, {}).get("frame")
    if frame:
        chunk, head = frame
        return np.arange(n, dtype=np.int64) * chunk + head, n * chunk
    offs = np.zeros(n, dtype=np.int64)
    if n:
        offs[1:] = np.cumsum(sizes[:-1])
    return offs, int(sizes.sum()) if n else 0


def build_batch(name: str, start: int, n: int, hdr: int = 64):
    """Host batch for packets [start, start+n): (umem uint8, descs structured) with packets packed
    back to back (a compacted AF_XDP UMEM / pcap-style buffer) or in frames (packet_offsets); bytes past
    `hdr` are zero."""
    from ._native import np_dtypes
    d_desc, _, _ = np_dtypes()
    idx = np.arange(start, start + n, dtype=np.uint64)
    sizes = packet_sizes(name, idx)
    offs, total = packet_offsets(name, sizes)
    umem = np.zeros(max(total, 1), dtype=np.uint8)
    h = headers(name, idx, hdr)
    if n:
        if np.all(sizes == sizes[0]) and sizes[0] >= hdr and not CONFIGS.get(name, {}).get("frame"):
            umem[:total].reshape(n, int(sizes[0]))[:, :hdr] = h
        else:
            cols = np.arange(hdr, dtype=np.int64)[None, :]
            for c0 in range(0, n, 1 << 20):  # chunked scatter of the header rows
                c1 = min(n, c0 + (1 << 20))
                pos = offs[c0:c1, None] + cols
                keep = cols < sizes[c0:c1, None]
                umem[pos[keep]] = h[c0:c1][keep]
    descs = np.zeros(n, dtype=d_desc)
    descs["addr"] = offs
    descs["len"] = sizes
    return umem, descs


def setup_vm(vm, name: str) -> int:
    """Load the config's maps (+ preloaded entries) and program into a VM; returns the program idx."""
    for mdef, entries in workload_maps(name):
        m = vm.add_map(mdef)
        if entries is not None:
            keys, vals = entries
            vm.map_update_batch(m, keys, vals)
    prog = vm.add_raw_program(CONFIGS[name]["program"]())
    vm.set_entrypoint(prog)
    return prog
