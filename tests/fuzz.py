"""Random-program generator for differential tests (oracle vs host simulation vs device).

Programs are raw eBPF slots biased toward the emulator's interesting paths: typed registers and
pointer arithmetic (ctx/packet/stack/map-value pointers), ValueMemory aliasing on the stack,
packet loads/stores, map helpers with stack keys, atomics, 32/64-bit ALU with edge immediates,
signed/unsigned jumps (forward, plus occasional back edges under a step budget), and illegal
registers / out-of-range jump targets that end in VM errors. Every run is deterministic in `seed`.
"""
from __future__ import annotations

import numpy as np

from gobpfld_amd.asm import (ADD, ALU, ALU64, AND, ARSH, ATOMIC, CALL, DIV, DW, EXIT, JEQ, JGE,
                             JGT, JMP, JMP32, JNE, JSGE, JSGT, JSLE, JSLT, LDX, LSH, MEM, MOD, MOV,
                             MUL, NEG, OR, RSH, ST, STX, SUB, XOR, B, H, K, W, X, raw)
from gobpfld_amd.emulator import MAP_ARRAY, MAP_HASH, MapDef, Settings

SIZES = [B, H, W, DW]
ALU_OPS = [ADD, SUB, MUL, DIV, OR, AND, LSH, RSH, MOD, XOR, MOV, ARSH]
JMP_OPS = [JEQ, JGT, JGE, JNE, JSGT, JSGE, JSLT, JSLE]
EDGE_IMMS = [0, 1, -1, 2, 7, 8, 14, 23, 31, 32, 63, 64, 0x7FFFFFFF, -0x80000000, 0xFF, 0xFFFF]

MAPS = [
    (MapDef(MAP_ARRAY, 4, 8, 16), None),
    (MapDef(MAP_HASH, 16, 16, 64), None),
    (MapDef(MAP_ARRAY, 4, 16, 4), None),
]


def _entries(rng):
    ents = {1: []}
    for _ in range(int(rng.integers(0, 12))):
        k = rng.integers(0, 4, size=16, dtype=np.uint8).tobytes()
        v = rng.integers(0, 256, size=16, dtype=np.uint8).tobytes()
        ents[1].append((k, v))
    return ents


def _reg(rng, allow_bad=True):
    """R0-R9 mostly; R10 (readable only through Copy, registers.go:90-114) and R11+ rarely."""
    r = int(rng.integers(0, 10))
    x = rng.random()
    if allow_bad and x < 0.025:
        r = 10
    elif allow_bad and x < 0.03:
        r = 11 + int(rng.integers(0, 5))
    return r


def gen_program(seed: int, length: int = 48):
    """-> (raw slots, maps, entries, settings)"""
    rng = np.random.default_rng(seed)
    p: list[int] = []
    # prologue: packet pointers, a stack key, a map lookup with a null check
    p += [raw(LDX | MEM | W, 2, 1, 0), raw(LDX | MEM | W, 3, 1, 4), raw(ALU64 | MOV | X, 6, 1)]
    if rng.random() < 0.7:
        p += [raw(ST | MEM | W, 10, 0, -4, int(rng.integers(0, 20))),
              raw(ST | MEM | W, 10, 0, -16, int(rng.integers(0, 3))),
              raw(ST | MEM | W, 10, 0, -12, 0), raw(ST | MEM | DW, 10, 0, -8, 0)]
        m = int(rng.integers(1, 4))
        key_off = -16 if m == 2 else -4
        p += [raw(0x18, 1, 1, 0, m), raw(0, 0, 0, 0, 0), raw(ALU64 | MOV | X, 2, 10),
              raw(ALU64 | ADD | K, 2, 0, 0, key_off), raw(JMP | CALL, 0, 0, 0, 1), raw(ALU64 | MOV | X, 7, 0)]
        p += [raw(JMP | JEQ | K, 0, 0, 2, 0), raw(LDX | MEM | DW, 8, 0, 0), raw(ALU64 | MOV | X, 9, 0)]
        # restore the packet pointers clobbered by the call (R1-R5 are caller-saved)
        p += [raw(LDX | MEM | W, 2, 6, 0), raw(LDX | MEM | W, 3, 6, 4)]
    body_start = len(p)
    n = int(rng.integers(length // 2, length))
    back_edges = rng.random() < 0.2
    for i in range(n):
        pc = len(p)
        c = rng.random()
        if c < 0.22:  # ALU
            op = ALU_OPS[int(rng.integers(len(ALU_OPS)))]
            cls = ALU64 if rng.random() < 0.7 else ALU
            if rng.random() < 0.5:
                imm = EDGE_IMMS[int(rng.integers(len(EDGE_IMMS)))] if rng.random() < 0.6 else int(rng.integers(-100, 100))
                p.append(raw(cls | op | K, _reg(rng), 0, 0, imm))
            else:
                p.append(raw(cls | op | X, _reg(rng), _reg(rng)))
        elif c < 0.27:
            p.append(raw((ALU64 if rng.random() < 0.5 else ALU) | NEG, _reg(rng)))
        elif c < 0.30:
            p.append(raw(ALU | 0xD0 | (X if rng.random() < 0.5 else K), _reg(rng), 0, 0,
                         [16, 32, 64][int(rng.integers(3))]))
        elif c < 0.40:  # pointer arithmetic on a packet/stack pointer
            d = [2, 10, 6, 7, 8][int(rng.integers(5))] if rng.random() < 0.8 else _reg(rng)
            dst = int(rng.integers(0, 10))
            p += [raw(ALU64 | MOV | X, dst, d), raw(ALU64 | ADD | K, dst, 0, 0, int(rng.integers(-24, 70)))]
        elif c < 0.55:  # loads
            s = SIZES[int(rng.integers(4))]
            src = [2, 10, 6, 7, 0][int(rng.integers(5))] if rng.random() < 0.7 else _reg(rng)
            off = int(rng.integers(-8, 48)) if src != 10 else -int(rng.integers(1, 40))
            p.append(raw(LDX | MEM | s, _reg(rng), src, off))
        elif c < 0.68:  # stores
            s = SIZES[int(rng.integers(4))]
            dst = [2, 10, 7, 0][int(rng.integers(4))] if rng.random() < 0.8 else _reg(rng)
            off = int(rng.integers(-8, 64)) if dst != 10 else -int(rng.integers(1, 40))
            if rng.random() < 0.5:
                p.append(raw(ST | MEM | s, dst, 0, off, int(rng.integers(-300, 300))))
            else:
                p.append(raw(STX | MEM | s, dst, _reg(rng), off))
        elif c < 0.72:  # atomics (ADD only translates; fetch form sometimes)
            s = DW if rng.random() < 0.5 else W
            dst = [7, 10, 2][int(rng.integers(3))]
            off = -8 if dst == 10 else int(rng.integers(0, 16))
            p.append(raw(STX | ATOMIC | s, dst, _reg(rng), off, 1 if rng.random() < 0.3 else 0))
        elif c < 0.88:  # conditional jumps
            op = JMP_OPS[int(rng.integers(len(JMP_OPS)))]
            cls = JMP if rng.random() < 0.7 else JMP32
            if back_edges and rng.random() < 0.25:
                off = -int(rng.integers(1, max(2, pc - body_start + 1)))
            else:
                off = int(rng.integers(0, 12))
            if rng.random() < 0.5:
                p.append(raw(cls | op | K, _reg(rng), 0, off, EDGE_IMMS[int(rng.integers(len(EDGE_IMMS)))]))
            else:
                p.append(raw(cls | op | X, _reg(rng), _reg(rng), off))
        elif c < 0.92:  # helpers (lookup/update/delete/smp-id, and an unknown id)
            h = [1, 2, 3, 14, 8, 1][int(rng.integers(6))]
            m = int(rng.integers(1, 4))
            p += [raw(0x18, 1, 1, 0, m), raw(0, 0, 0, 0, 0), raw(ALU64 | MOV | X, 2, 10),
                  raw(ALU64 | ADD | K, 2, 0, 0, -16 if m == 2 else -4)]
            if h == 2:
                p += [raw(ALU64 | MOV | X, 3, 10), raw(ALU64 | ADD | K, 3, 0, 0, -32),
                      raw(ST | MEM | DW, 10, 0, -32, int(rng.integers(0, 9))), raw(ST | MEM | DW, 10, 0, -24, 1),
                      raw(ALU64 | MOV | K, 4, 0, 0, int(rng.integers(0, 3)))]
            p.append(raw(JMP | CALL, 0, 0, 0, h))
        elif c < 0.94:
            p += [raw(0x18, _reg(rng, False), 0, 0, int(rng.integers(-2**31, 2**31))), raw(0, 0, 0, 0, int(rng.integers(-2**31, 2**31)))]
        elif c < 0.96:
            p.append(raw(JMP | 0x00, 0, 0, int(rng.integers(0, 6))))  # ja
        else:
            p.append(raw(ALU64 | MOV | K, 0, 0, 0, int(rng.integers(0, 5))))
            p.append(raw(JMP | EXIT))
    p.append(raw(ALU64 | MOV | K, 0, 0, 0, 2))
    p.append(raw(JMP | EXIT))
    # occasionally a target past the end (BAD_PC fallthrough) is left in by the jumps above
    settings = Settings(max_steps=int(rng.integers(200, 2000)) if back_edges else 0)
    return p, list(MAPS), _entries(rng), settings


# ---------------------------------------------------------------------------------------------------
# Ordered maps: LRU_HASH, QUEUE, STACK, PERF_EVENT_ARRAY (and a HASH beside them)
#
# Programs are sequences of map operations on keys taken from packet bytes (small masks make hot keys),
# with IMM key / value registers now and then (errMapKeyNoPtr / errMapValNoPtr after an eviction,
# maps_hash_lru.go:113-137), value reads / adds / stores through returned pointers, pops and peeks read
# back, perf outputs of packet or stack bytes, forward branches on packet bytes between operations, and
# starting states that are empty, partly full or full. They drive the keyed path, the parallel list
# operations (count pass, pop ranks), LRU stamps and the one-lane replay's order log, and the decisions
# between them (tests/test_fuzz_ordered.py).
# ---------------------------------------------------------------------------------------------------
ORD_LRU, ORD_QUEUE, ORD_STACK, ORD_PERF, ORD_HASH = 1, 2, 3, 4, 5
_KEY_MASKS = [1, 3, 7, 15, 63, 255]


def gen_ordered_program(seed: int):
    """-> (raw slots, maps, entries, settings) for an ordered-map program."""
    from gobpfld_amd.asm import JGT, Asm
    from gobpfld_amd.emulator import MAP_LRU_HASH, MAP_PERF_EVENT_ARRAY, MAP_QUEUE, MAP_STACK
    rng = np.random.default_rng(seed + 1_000_003)
    lru_max = int(rng.choice([4, 8, 16, 64]))
    list_max = int(rng.choice([4, 16, 64]))
    maps = [(MapDef(MAP_LRU_HASH, 4, 8, lru_max), None),
            (MapDef(MAP_QUEUE, 0, 8, list_max), None),
            (MapDef(MAP_STACK, 0, 8, list_max), None),
            (MapDef(MAP_PERF_EVENT_ARRAY, 4, 4, 8), None),
            (MapDef(MAP_HASH, 4, 8, 32), None)]
    ents = {}
    fill = rng.choice(["empty", "part", "full"], p=[0.2, 0.35, 0.45])
    nl = {"empty": 0, "part": int(rng.integers(1, lru_max)), "full": lru_max}[fill]
    lkeys = rng.permutation(256)[:nl] if rng.random() < 0.5 else np.arange(nl)
    ents[0] = [(int(k).to_bytes(4, "little"), rng.integers(0, 256, size=8, dtype=np.uint8).tobytes()) for k in lkeys]
    for i in (1, 2):
        ents[i] = [(None, rng.integers(0, 256, size=8, dtype=np.uint8).tobytes())
                   for _ in range(int(rng.integers(0, list_max + 1)))]
    ents[4] = [(int(k).to_bytes(4, "little"), rng.integers(0, 256, size=8, dtype=np.uint8).tobytes())
               for k in rng.permutation(64)[:int(rng.integers(0, 20))]]

    a = Asm()
    a.ldx(4, 6, 1, 0).ldx(4, 7, 1, 4)
    a.mov64(2, src=6).add64(2, 16)
    a.jmp(JGT, 2, "short", src=7)  # the packet must hold 16 bytes
    a.mov64(9, 0)
    a.st(8, 10, -32, 0).st(8, 10, -40, 0)
    labels = 0

    def key(off):
        """stack key at r10-4 = packet[off] & mask (or a constant); R2 = its pointer (or an IMM)."""
        if rng.random() < 0.85:
            a.ldx(1, 3, 6, off).alu64(AND, 3, int(_KEY_MASKS[int(rng.integers(len(_KEY_MASKS)))]))
            a.stx(4, 10, -4, 3)
        else:
            a.st(4, 10, -4, int(rng.integers(0, 8)))
        if rng.random() < 0.04:
            a.mov64(2, int(rng.integers(0, 5)))  # an IMM key
        else:
            a.mov64(2, src=10).add64(2, -4)

    def value():
        """R3 = a pointer to 8 value bytes at r10-16 (packet bytes or a constant), or an IMM."""
        if rng.random() < 0.12:
            a.mov64(3, int(rng.integers(0, 3)))
            return
        if rng.random() < 0.5:
            a.ldx(8, 3, 6, int(rng.integers(0, 9))).stx(8, 10, -16, 3)
        else:
            a.st(8, 10, -16, int(rng.integers(-5, 50)))
        a.mov64(3, src=10).add64(3, -16)

    nops = int(rng.integers(1, 7))
    pending_skip = None
    # profiles: every operation, LRU / HASH only (the keyed path's inserts, evictions, value stores), or
    # lists and perf outputs only (count pass, pop ranks, appends)
    profile = rng.choice(["mixed", "keys", "lists"], p=[0.5, 0.3, 0.2])
    for i in range(nops):
        if pending_skip:
            a.label(pending_skip)
            pending_skip = None
        c = rng.random()
        if profile == "keys":
            c = c * 0.58 if c < 0.9 else 0.96
        elif profile == "lists":
            c = 0.58 + c * 0.42
        off = int(rng.integers(0, 16))
        if c < 0.25:  # LRU / HASH lookup, then use the value
            m = ORD_LRU if rng.random() < 0.8 else ORD_HASH
            a.ld_map(1, m)
            key(off)
            a.call(1)
            labels += 1
            miss = f"miss{labels}"
            a.jmp(JEQ, 0, miss, imm=0)
            u = rng.random()
            if u < 0.35:
                a.ldx(8, 5, 0, 0).alu64(ADD, 9, src=5)
            elif u < 0.6:
                a.mov64(1, int(rng.integers(1, 4))).xadd(8, 0, 0, 1)
            elif u < 0.8:
                a.stx(8, 0, 0, 9)  # a plain store into the value: a map-entry write (keyed)
            a.label(miss)
        elif c < 0.5:  # update
            m = ORD_LRU if rng.random() < 0.85 else ORD_HASH
            a.ld_map(1, m)
            key(off)
            value()
            a.mov64(4, int(rng.choice([0, 0, 0, 1, 2])))
            a.call(2).alu64(ADD, 9, src=0)
        elif c < 0.58:  # delete
            m = ORD_LRU if rng.random() < 0.8 else ORD_HASH
            a.ld_map(1, m)
            key(off)
            a.call(3).alu64(ADD, 9, src=0)
        elif c < 0.72:  # push
            m = ORD_QUEUE if rng.random() < 0.5 else ORD_STACK
            a.ld_map(1, m)
            value()
            a.mov64(2, src=3).mov64(3, int(rng.choice([0, 0, 2])))
            a.call(87).alu64(ADD, 9, src=0)
        elif c < 0.82:  # pop, and read the element back
            m = ORD_QUEUE if rng.random() < 0.5 else ORD_STACK
            a.ld_map(1, m).mov64(2, src=10).add64(2, -32)
            a.call(88).alu64(ADD, 9, src=0)
            labels += 1
            a.ldx(8, 3, 10, -32)
            a.jmp(JEQ, 3, f"nopop{labels}", imm=0)
            a.ldx(8, 5, 3, 0).alu64(ADD, 9, src=5)
            a.label(f"nopop{labels}")
        elif c < 0.88:  # peek
            m = ORD_QUEUE if rng.random() < 0.5 else ORD_STACK
            a.ld_map(1, m).mov64(2, src=10).add64(2, -40)
            a.call(89)
            labels += 1
            a.jmp(JNE, 0, f"nopeek{labels}", imm=0)
            a.ldx(8, 5, 2, 0).alu64(ADD, 9, src=5)
            a.label(f"nopeek{labels}")
        elif c < 0.95:  # perf output of packet bytes or of the stack
            a.ld_map(2, ORD_PERF).mov64(3, 0)
            if rng.random() < 0.7:
                a.mov64(4, src=6).add64(4, int(rng.integers(0, 8)))
            else:
                a.mov64(4, src=10).add64(4, -16).st(8, 10, -16, int(rng.integers(0, 99)))
            if rng.random() < 0.5:
                a.ldx(1, 5, 6, off).alu64(AND, 5, 7).add64(5, 1)
            else:
                a.mov64(5, int(rng.choice([0, 4, 8])))
            a.call(25).alu64(ADD, 9, src=0)
        else:  # skip the next operation on a packet bit
            labels += 1
            pending_skip = f"skip{labels}"
            a.ldx(1, 4, 6, off).alu64(AND, 4, int(rng.choice([1, 2, 4])))
            a.jmp(JNE, 4, pending_skip, imm=0)
    if pending_skip:
        a.label(pending_skip)
    a.mov64(0, src=9)
    if rng.random() < 0.5:
        a.alu64(AND, 0, 3)
    a.exit()
    a.label("short").mov64(0, 1).exit()
    return a.assemble(), maps, ents, Settings()


def ordered_packets(seed: int, n: int):
    """n packets of 8-64 bytes (a few shorter than the programs' 16), bytes from a small alphabet so
    that packets share keys."""
    from gobpfld_amd._native import np_dtypes
    d_desc, _, _ = np_dtypes()
    rng = np.random.default_rng(seed ^ 0x0DDE)
    lens = rng.choice([8, 16, 20, 32, 64], size=n, p=[0.03, 0.3, 0.27, 0.2, 0.2])
    offs = (np.arange(n) * 64).astype(np.int64)
    alpha = int(rng.choice([4, 16, 256]))
    umem = rng.integers(0, alpha, size=n * 64, dtype=np.uint8)
    descs = np.zeros(n, dtype=d_desc)
    descs["addr"] = offs
    descs["len"] = lens
    return umem, descs
