"""Packet ingestion: pcap records into AF_XDP-shaped UMEM frames and descriptors
(include/xdpemu_io.h, gobpfld_amd/xsk.py), the XSK ring semantics of xsk.go, and the programs run
on what the queue posts: oracle vs host simulation on CPU, the streaming device path on the GPU.
The capture files are written here (tests hold no pcap fixtures of the reference; its XSK code needs
kernel sockets, so its behaviour is restated from xsk.go and checked through these properties)."""
import struct

import numpy as np
import pytest

from gobpfld_amd import workloads as W
from gobpfld_amd import xsk as X
from gobpfld_amd.emulator import VM, Settings
from parity import packets


def _pkts(n, seed=3):
    rng = np.random.default_rng(seed)
    sizes = rng.choice([14, 60, 64, 128, 577, 1514], size=n)
    return [rng.integers(0, 256, size=int(s), dtype=np.uint8).tobytes() for s in sizes]


@pytest.mark.parametrize("ns,be", [(False, False), (True, False), (False, True), (True, True)])
def test_pcap_formats_fill_frames(built, ns, be):
    pk = _pkts(50)
    ts = np.arange(50, dtype=np.uint64) * np.uint64(1_000_001_000) + np.uint64(7_000)
    pc = X.PcapFile(X.write_pcap(None, pk, ts_ns=ts, nanosecond=ns, big_endian=be))
    assert (pc.info.nanosecond, pc.info.swapped, pc.info.linktype) == (int(ns), int(be), 1)
    assert pc.count() == (50, sum(map(len, pk)))
    umem = np.zeros(64 * 2048, np.uint8)
    frames = np.arange(50, dtype=np.uint64)[::-1] * np.uint64(2048)     # any frame order
    desc, olen, got_ts = pc.fill(umem, 2048, 256, frames, want_meta=True)
    assert len(desc) == 50 and pc.count() == (0, 0)
    assert (desc["addr"] == frames + np.uint64(256)).all() and (desc["options"] == 0).all()
    assert (olen == [len(p) for p in pk]).all()
    assert (got_ts == ts).all()
    for d, p in zip(desc, pk):
        assert umem[int(d["addr"]):int(d["addr"]) + int(d["len"])].tobytes() == p


def test_pcap_truncation_and_bad_input(built):
    pk = [bytes(range(200)) * 10, b"\x01" * 60]                          # 2000 B does not fit 2048 - 512
    data = X.write_pcap(None, pk)
    pc = X.PcapFile(data + data[24:24 + 16 + 10])                       # plus a cut-off third record
    assert pc.count()[0] == 2
    umem = np.zeros(4 * 2048, np.uint8)
    desc, olen, _ = pc.fill(umem, 2048, 512, np.array([0, 2048, 4096], np.uint64), want_meta=True)
    assert list(desc["len"]) == [1536, 60] and list(olen) == [2000, 60]
    assert umem[512:512 + 1536].tobytes() == pk[0][:1536]
    assert pc.offset == len(data)                                      # the cut-off record stays unread
    with pytest.raises(X.XSKError, match="not a classic pcap"):
        X.PcapFile(b"\0" * 64)
    with pytest.raises(X.XSKError, match="not a classic pcap"):
        X.PcapFile(data[:20])
    with pytest.raises(X.XSKError, match="link type"):
        X.PcapFile(data[:20] + struct.pack("<I", 101) + data[24:])
    pc.rewind()
    with pytest.raises(X.XSKError, match="outside the UMEM"):
        pc.fill(umem, 2048, 0, np.array([4 * 2048], np.uint64))
    empty = X.PcapFile(data[:24])
    assert empty.count() == (0, 0) and len(empty.fill(umem, 2048, 0, np.array([0], np.uint64))) == 0


def test_pcap_pack_alignment_and_capacity(built):
    pk = _pkts(40, seed=5)
    pc = X.PcapFile(X.write_pcap(None, pk))
    d_desc = X.N.np_dtypes()[0]
    buf = np.zeros(6000, np.uint8)
    desc = np.zeros(64, d_desc)
    n, used = pc.pack(buf, desc, align=64)
    assert 0 < n < 40 and used <= buf.size
    assert (desc["addr"][:n] % 64 == 0).all()
    assert (np.diff(desc["addr"][:n].astype(np.int64)) == (-(-desc["len"][:n - 1].astype(np.int64) // 64) * 64)).all()
    for d, p in zip(desc[:n], pk):
        assert buf[int(d["addr"]):int(d["addr"]) + int(d["len"])].tobytes() == p
    rest = 0
    while True:                                                        # the rest follows on later calls
        k, _ = pc.pack(buf, desc, align=64, max_len=100)
        if not k:
            break
        assert (desc["len"][:k] <= 100).all()
        rest += k
    assert n + rest == 40


def test_ring_semantics():
    r = X.AddrRing(8)
    for i in range(7):
        r.enqueue(i)
    with pytest.raises(X.RingFull):                                    # full one slot early (xsk.go:590)
        r.enqueue(7)
    assert [int(r.dequeue()) for _ in range(7)] == list(range(7)) and r.dequeue() is None
    r.producer = r.consumer = 0xFFFFFFFE                               # u32 wraparound of the indices
    r.enqueue_many(np.arange(5, dtype=np.uint64))
    assert len(r) == 5 and r.producer == 3
    assert list(r.dequeue_many(10)) == list(range(5)) and len(r) == 0
    with pytest.raises(X.XSKError):
        X.DescRing(6)


def test_settings_checks_and_queue_layout():
    for bad, msg in [(dict(FrameCount=3000), "power of 2"), (dict(FrameSize=1000), "2048 or 4096"),
                     (dict(DisableTx=True, DisableRx=True), "both be disabled")]:
        with pytest.raises(X.XSKError, match=msg):
            X.XSKSettings(**bad).validated()
    q = X.XSKQueue(X.XSKSettings(FrameSize=2048, FrameCount=16, Headroom=128))
    assert (q.rx_count, q.tx_count) == (8, 8) and len(q.fill) == 7    # rxCount - 1 frames (xsk.go:1026)
    assert sorted(int(a) for a in q.tx_free) == [2048 * i for i in range(8, 16)]
    assert X.XSKSettings(DisableTx=True).validated().counts() == (4096, 0)


def test_queue_rx_recycle_tx(built):
    pk = _pkts(20, seed=9)
    pc = X.PcapFile(X.write_pcap(None, pk))
    q = X.XSKQueue(X.XSKSettings(FrameSize=2048, FrameCount=16, Headroom=64))
    assert q.receive(pc, 100) == 7                                     # bounded by the fill ring
    desc = q.rx.dequeue_many(7)
    assert (desc["addr"] % 2048 == 64).all()
    q.transmit(desc[:2])
    assert len(q.tx_free) == 8                                         # completed at once
    q.recycle(desc)
    assert len(q.fill) == 7 and set(q.fill.dequeue_many(7) % np.uint64(2048)) == {0}


def _queue_batches(pk, lib):
    """All records through an XSK queue: the (umem, rx descriptors) batches a program would see."""
    pc = X.PcapFile(X.write_pcap(None, pk))
    q = X.XSKQueue(X.XSKSettings(FrameSize=2048, FrameCount=64, Headroom=256))
    out = []
    while True:
        n = q.receive(pc, 16)
        if not n:
            break
        desc = q.rx.dequeue_many(n)
        out.append((q.umem.copy(), desc))
        q.recycle(desc)
    return out


def _run_cfg(lib, batches, name="c2"):
    vm = VM(Settings(), lib=lib)
    W.setup_vm(vm, name)
    ver = np.concatenate([vm.run_batch(u, d).verdicts for u, d in batches])
    dump = [vm.map_dump(m) for m in range(1, 1 + len(W.workload_maps(name)))]
    vm.close()
    return ver, dump


def test_queue_batches_oracle_equal_hostsim(oracle_lib, hostsim_lib):
    umem, descs = W.build_batch("c2", 0, 300)
    pk = [umem[int(d["addr"]):int(d["addr"]) + int(d["len"])].tobytes() for d in descs]
    batches = _queue_batches(pk, oracle_lib)
    v_o, m_o = _run_cfg(oracle_lib, batches)
    v_h, m_h = _run_cfg(hostsim_lib, batches)
    assert (v_o == v_h).all() and m_o == m_h
    # the frames + headroom layout changes nothing against the packed batch
    vm = VM(Settings(), lib=oracle_lib)
    W.setup_vm(vm, "c2")
    assert (vm.run_batch(umem.copy(), descs).verdicts == v_o).all()
    vm.close()


@pytest.mark.gpu
def test_run_pcap_device_equals_oracle(gpu_lib, oracle_lib, tmp_path):
    n = 200_000
    umem, descs = W.build_batch("c2", 0, n)
    pk = [umem[int(d["addr"]):int(d["addr"]) + int(d["len"])].tobytes() for d in descs]
    path = tmp_path / "c2.pcap"
    X.write_pcap(path, pk)
    vm = VM(Settings(), lib=gpu_lib)
    W.setup_vm(vm, "c2")
    pc = X.PcapFile(path)
    res = X.run_pcap(vm, pc, batch=1 << 16, keep_verdicts=True)
    dev_maps = [vm.map_dump(m) for m in range(1, 1 + len(W.workload_maps("c2")))]
    vm.close()
    pc.close()
    ref = VM(Settings(), lib=oracle_lib)
    W.setup_vm(ref, "c2")
    want = ref.run_batch(umem.copy(), descs)
    ref_maps = [ref.map_dump(m) for m in range(1, 1 + len(W.workload_maps("c2")))]
    ref.close()
    assert res.packets == n and res.batches == 4 and res.status_count[0] == n
    assert (res.verdicts == want.verdicts).all()
    assert dev_maps == ref_maps
    assert sum(res.verdict_count.values()) == n
