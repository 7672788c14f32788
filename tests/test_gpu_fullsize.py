"""Full-size parity through size-independent properties (-m gpu): per-flow counters and verdicts of the
HASH configs at BASELINE batch sizes, against truth computed from the generated flows with numpy
(no emulator involved), plus the "a second identical run doubles every counter" property."""
import numpy as np
import pytest

from gobpfld_amd import workloads as W
from gobpfld_amd.emulator import VM, Settings

pytestmark = pytest.mark.gpu


def _device_run(name, n, runs=1):
    import torch
    umem, descs = W.build_batch(name, 0, n)
    vm = VM(Settings())
    W.setup_vm(vm, name)
    d_umem = torch.from_numpy(umem).cuda()
    d_desc = torch.from_numpy(descs.view(np.uint8)).cuda()
    d_ver = torch.zeros(n, dtype=torch.int32, device="cuda")
    dumps, stats = [], []
    for _ in range(runs):
        st = vm.run_batch_device(d_umem.data_ptr(), d_umem.numel(), d_desc.data_ptr(), n, d_verdicts=d_ver.data_ptr())
        torch.cuda.synchronize()
        stats.append(st)
        dumps.append(vm.map_dump(1))
    ver = d_ver.cpu().numpy().view(np.uint32)
    vm.close()
    return ver, dumps, stats


def _sorted_by_key(keys: np.ndarray, vals: np.ndarray):
    """Rows ordered by key bytes (xe_map_dump order)."""
    o = np.lexsort(keys.T[::-1])  # byte 0 is the primary sort key (memcmp order)
    return keys[o], vals[o]


def test_c5_fullsize_per_flow_counters():
    n = 16 * 1024 * 1024
    idx = np.arange(n, dtype=np.uint64)
    fid = W.rng_stream(5, idx, 0) % np.uint64(W.C5_FLOWS + W.C5_FLOWS // 16)
    hit = fid < np.uint64(W.C5_FLOWS)
    pkts = np.bincount(fid[hit].astype(np.int64), minlength=W.C5_FLOWS).astype(np.uint64)
    keys, _ = W.c5_map_entries()
    vals = np.zeros((W.C5_FLOWS, 2), dtype=np.uint64)
    vals[:, 0] = pkts
    vals[:, 1] = pkts * np.uint64(64)
    want_k, want_v = _sorted_by_key(keys, vals)
    ver, dumps, stats = _device_run("c5", n, runs=2)
    assert stats[0]["status_count"][0] == n and stats[0]["conflict"] == 0 and stats[0]["mode_used"] == 1
    assert (ver == 2).all()                                            # every C5 packet is IPv4: PASS
    for r, (k, v) in enumerate(dumps, start=1):
        assert np.array_equal(np.asarray(k).reshape(-1, 16), want_k)
        got = np.frombuffer(np.asarray(v).tobytes(), dtype=np.uint64).reshape(-1, 2)
        assert np.array_equal(got, want_v * np.uint64(r)), f"run {r}: per-flow {{pkts, bytes}} differ"


def test_c3_fullsize_redirect_and_hits():
    n = 4 * 1024 * 1024
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
    ver, dumps, stats = _device_run("c3", n)
    assert stats[0]["status_count"][0] == n and stats[0]["conflict"] == 0
    assert (ver == np.where(hit, 4, 2)).all()                          # REDIRECT on a hit, PASS on a miss
    k, v = dumps[0]
    assert np.array_equal(np.asarray(k).reshape(-1, 16), want_k)
    got = np.frombuffer(np.asarray(v).tobytes(), dtype=np.uint64).reshape(-1, 2)
    assert np.array_equal(got, want_v), "per-flow {flow_id, hits} differ"
