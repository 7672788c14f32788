"""Full-size parity at the BASELINE batch sizes the bench times (-m gpu).

Every BASELINE workload is checked at the size `bench.py` measures it, through properties that do
not depend on the size: per-packet verdicts and per-flow / per-proto counters against truth computed
from the generated headers with numpy (no emulator involved), "a second identical run doubles every
counter", a keyed learning batch against one sequential oracle VM (the reference's per-packet loop,
emulator/vm.go:110-173), and determinism under permuted chunk -> wave schedules.

Batches are built on the device (headers scattered into a zeroed UMEM) so a 16M x 1500 B batch needs no
25 GB host buffer.
"""
import numpy as np
import pytest

from gobpfld_amd import workloads as W
from gobpfld_amd.emulator import MODE_KEYED, MODE_PARALLEL, VM, Settings

pytestmark = pytest.mark.gpu
N16M = 16 * 1024 * 1024


def _device_batch(name, n, start=0):
    """(d_umem, d_desc, host headers) of packets [start, start + n) of config `name`, packed back to back
    exactly as workloads.build_batch lays them out; bytes past the 64-byte header are zero."""
    import torch
    from gobpfld_amd._native import np_dtypes
    idx = np.arange(start, start + n, dtype=np.uint64)
    sizes = W.packet_sizes(name, idx)
    assert sizes.min() >= 64
    offs = np.zeros(n, dtype=np.int64)
    offs[1:] = np.cumsum(sizes[:-1])
    total = int(sizes.sum())
    h = W.headers(name, idx, 64)
    d_umem = torch.zeros(total, dtype=torch.uint8, device="cuda")
    cols = torch.arange(64, device="cuda", dtype=torch.int64)
    step = 1 << 21
    for c0 in range(0, n, step):
        c1 = min(n, c0 + step)
        pos = torch.from_numpy(offs[c0:c1]).cuda()[:, None] + cols
        d_umem[pos.reshape(-1)] = torch.from_numpy(h[c0:c1]).cuda().reshape(-1)
    d_desc_t, _, _ = np_dtypes()
    descs = np.zeros(n, dtype=d_desc_t)
    descs["addr"] = offs
    descs["len"] = sizes
    d_desc = torch.from_numpy(descs.view(np.uint8)).cuda()
    torch.cuda.synchronize()
    return d_umem, d_desc, h, sizes


def _device_run(name, n, runs=1, sched=0, batch=None):
    import torch
    d_umem, d_desc, h, sizes = batch or _device_batch(name, n)
    vm = VM(Settings())
    W.setup_vm(vm, name)
    if sched:
        vm.set_schedule(sched)
    vm.prepare()
    d_ver = torch.zeros(n, dtype=torch.int32, device="cuda")
    dumps, stats = [], []
    for _ in range(runs):
        st = vm.run_batch_device(d_umem.data_ptr(), d_umem.numel(), d_desc.data_ptr(), n, d_verdicts=d_ver.data_ptr())
        torch.cuda.synchronize()
        stats.append(st)
        dumps.append(vm.map_dump(1) if W.workload_maps(name) else None)
    ver = d_ver.cpu().numpy().view(np.uint32)
    vm.close()
    return ver, dumps, stats


def _sorted_by_key(keys: np.ndarray, vals: np.ndarray):
    """Rows ordered by key bytes (xe_map_dump order)."""
    o = np.lexsort(keys.T[::-1])  # byte 0 is the primary sort key (memcmp order)
    return keys[o], vals[o]


def _c5_truth(n):
    idx = np.arange(n, dtype=np.uint64)
    fid = W.rng_stream(5, idx, 0) % np.uint64(W.C5_FLOWS + W.C5_FLOWS // 16)
    hit = fid < np.uint64(W.C5_FLOWS)
    pkts = np.bincount(fid[hit].astype(np.int64), minlength=W.C5_FLOWS).astype(np.uint64)
    keys, _ = W.c5_map_entries()
    vals = np.zeros((W.C5_FLOWS, 2), dtype=np.uint64)
    vals[:, 0] = pkts
    vals[:, 1] = pkts * np.uint64(64)
    return _sorted_by_key(keys, vals)


def test_c5_fullsize_per_flow_counters():
    """C5's per-GPU shard of the bench (33,554,432 x 64 B, BASELINE configs[4] / 8): per-flow {pkts,
    bytes} equal the flow histogram of the generated stream, and a second run doubles them."""
    n = 2 * N16M
    want_k, want_v = _c5_truth(n)
    ver, dumps, stats = _device_run("c5", n, runs=2)
    assert stats[0]["status_count"][0] == n and stats[0]["conflict"] == 0 and stats[0]["mode_used"] == MODE_PARALLEL
    assert (ver == 2).all()                                            # every C5 packet is IPv4: PASS
    for r, (k, v) in enumerate(dumps, start=1):
        assert np.array_equal(np.asarray(k).reshape(-1, 16), want_k)
        got = np.frombuffer(np.asarray(v).tobytes(), dtype=np.uint64).reshape(-1, 2)
        assert np.array_equal(got, want_v * np.uint64(r)), f"run {r}: per-flow {{pkts, bytes}} differ"


def _c3_truth(n):
    idx = np.arange(n, dtype=np.uint64)
    r0 = W.rng_stream(3, idx, 0)
    u = (r0 >> np.uint64(11)).astype(np.float64) / float(1 << 53)
    hit = (W.rng_stream(3, idx, 2) % np.uint64(10)) != 0
    fid = W.zipf_ranks(u, W.C3_FLOWS)
    hits = np.bincount(fid[hit], minlength=W.C3_FLOWS).astype(np.uint64)
    keys, vals0 = W.c3_map_entries()
    vals = vals0.view(np.uint64).reshape(-1, 2).copy()
    vals[:, 1] = hits
    want_k, want_v = _sorted_by_key(keys, vals)
    return hit, want_k, want_v


def test_c3_fullsize_redirect_and_hits():
    """C3 at the bench's 16M IMIX packets: REDIRECT exactly on the preloaded flows, hits per flow."""
    n = N16M
    hit, want_k, want_v = _c3_truth(n)
    ver, dumps, stats = _device_run("c3", n)
    assert stats[0]["status_count"][0] == n and stats[0]["conflict"] == 0
    assert (ver == np.where(hit, 4, 2)).all()                          # REDIRECT on a hit, PASS on a miss
    k, v = dumps[0]
    assert np.array_equal(np.asarray(k).reshape(-1, 16), want_k)
    got = np.frombuffer(np.asarray(v).tobytes(), dtype=np.uint64).reshape(-1, 2)
    assert np.array_equal(got, want_v), "per-flow {flow_id, hits} differ"


def _c4_truth(h: np.ndarray) -> np.ndarray:
    """First-match over the 48 ACL rules, evaluated on the header bytes the program reads (IPv4 at 14:
    saddr u32 LE at 26, proto at 23, dport u16 LE at 36; JNE32 on saddr, JNE on proto, JGT on dport);
    no match (or not IPv4) -> DROP. workloads.prog_c4."""
    h64 = h.astype(np.uint64)
    ipv4 = (h[:, 12] == 0x08) & (h[:, 13] == 0x00)
    saddr = h64[:, 26] | (h64[:, 27] << 8) | (h64[:, 28] << 16) | (h64[:, 29] << 24)
    proto = h64[:, 23]
    dport = h64[:, 36] | (h64[:, 37] << 8)
    verdict = np.full(len(h), 1, dtype=np.uint32)                      # XDP_DROP
    open_ = ipv4.copy()
    for s_le, p, dmax, action in W.acl_rules():
        m = open_ & (saddr == np.uint64(s_le)) & (proto == np.uint64(p)) & (dport <= np.uint64(dmax))
        verdict[m] = action
        open_ &= ~m
    return verdict


def test_c4_fullsize_first_match():
    """C4 at the bench's 16M x 1500 B: every verdict is the first-matching rule's action."""
    n = N16M
    batch = _device_batch("c4", n)
    want = _c4_truth(batch[2])
    assert 0.3 < (want == 2).mean() < 0.7                              # both actions well represented
    ver, _, stats = _device_run("c4", n, batch=batch)
    assert stats[0]["status_count"][0] == n and stats[0]["mode_used"] == MODE_PARALLEL
    assert (ver == want).all(), f"{int((ver != want).sum())} verdicts differ"


@pytest.mark.parametrize("n", [4 * 1024 * 1024, N16M], ids=["4M", "16M"])
def test_c3learn_keyed_bench_size_equals_oracle(oracle_lib, n):
    """The bench's keyed side line (C3-learn, 4,194,304 IMIX packets whose misses insert their flow) and
    the 16M batch DESIGN.md quotes, through the keyed path, against one sequential oracle VM: results,
    verdicts and the final table."""
    import torch
    umem, descs = W.build_batch("c3learn", 0, n)
    ov = VM(Settings(), lib=oracle_lib)
    W.setup_vm(ov, "c3learn")
    ro = ov.run_batch(umem.copy(), descs)
    ok_, ov_ = ov.map_dump(1)
    ov.close()
    d_umem = torch.from_numpy(umem).cuda()
    d_desc = torch.from_numpy(descs.view(np.uint8)).cuda()
    d_res = torch.zeros(n * 16, dtype=torch.uint8, device="cuda")
    d_ver = torch.zeros(n, dtype=torch.int32, device="cuda")
    vm = VM(Settings())
    W.setup_vm(vm, "c3learn")
    vm.prepare()
    st = vm.run_batch_device(d_umem.data_ptr(), d_umem.numel(), d_desc.data_ptr(), n, d_results=d_res.data_ptr(),
                             d_verdicts=d_ver.data_ptr())
    torch.cuda.synchronize()
    assert st["mode_used"] == MODE_KEYED, st
    res = d_res.cpu().numpy().view(ro.results.dtype)
    bad = np.nonzero(res != ro.results)[0]
    assert len(bad) == 0, f"{len(bad)} results differ, first at {bad[0]}: {res[bad[0]]} vs {ro.results[bad[0]]}"
    assert (d_ver.cpu().numpy().view(np.uint32) == ro.verdicts).all()
    k, v = vm.map_dump(1)
    vm.close()
    assert len(k) == len(ok_) > W.C3_FLOWS
    assert np.array_equal(k, ok_) and np.array_equal(v, ov_), "learned flow table differs"
    assert st["steps"] == ro.stats["steps"]


@pytest.mark.parametrize("name", ["c3", "c5"])
def test_schedule_permutation_is_invisible(name):
    """Determinism: the same batch under permuted chunk -> wave schedules gives identical
    verdicts and identical map contents (hash counters added from every wave in a different order)."""
    n = 4 * 1024 * 1024
    batch = _device_batch(name, n)
    base_v, base_d, _ = _device_run(name, n, batch=batch)
    for sched in (1, 977, 123457):
        v, d, st = _device_run(name, n, sched=sched, batch=batch)
        assert st[0]["conflict"] == 0
        assert np.array_equal(v, base_v), f"schedule {sched}: verdicts differ"
        assert np.array_equal(d[0][0], base_d[0][0]) and np.array_equal(d[0][1], base_d[0][1]), f"schedule {sched}: map differs"
