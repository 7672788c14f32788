"""bench.py's self-check (`verified` in the bench line) compares the device with truth derived from the
generated headers (bench.shard_truth / expected_map). Pin that truth here against the CPU oracle — one
VM walking a shard twice, the reference's per-packet loop (emulator/vm.go:110-173) — so a wrong truth
cannot pass or fail the GPU run silently. Shards start past 0 (ranks k > 0)."""
import importlib.util
from pathlib import Path

import numpy as np
import pytest

from gobpfld_amd import workloads as W
from gobpfld_amd.emulator import VM, Settings

ROOT = Path(__file__).resolve().parent.parent


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", ROOT / "bench.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


@pytest.mark.parametrize("name,start,n", [("c1", 0, 512), ("c2", 3 * 4096, 4096), ("c3", 8192, 3000),
                                          ("c4", 5000, 2000), ("c5", 1 << 20, 3000)])
def test_shard_truth_equals_oracle(oracle_lib, name, start, n):
    B = _bench()
    want_v, delta = B.shard_truth(name, start, n)
    vm = VM(Settings(), lib=oracle_lib)
    W.setup_vm(vm, name)
    umem, descs = W.build_batch(name, start, n)
    for _ in range(2):
        r = vm.run_batch(umem.copy(), descs)
        assert (r.verdicts == want_v).all(), f"{name}: {int((r.verdicts != want_v).sum())} verdicts differ"
    if delta is not None:
        exp = B.expected_map(name, 2 * delta)
        got = vm.map_dump(1)
        if isinstance(exp, bytes):
            assert got == exp
        else:
            k, v = got
            assert np.array_equal(np.asarray(k), exp[0])
            assert np.array_equal(np.frombuffer(np.asarray(v).tobytes(), np.uint64).reshape(-1, 2), exp[1])
    vm.close()


def test_shard_truths_sum_over_ranks(oracle_lib):
    """Two shards' per-run effects summed equal one VM over both shards in order (what the exchange makes
    every replica hold)."""
    B = _bench()
    n = 2048
    tot = sum(B.shard_truth("c2", k * n, n)[1] for k in range(2))
    vm = VM(Settings(), lib=oracle_lib)
    W.setup_vm(vm, "c2")
    umem, descs = W.build_batch("c2", 0, 2 * n)
    vm.run_batch(umem, descs)
    assert vm.map_dump(1) == B.expected_map("c2", tot)
    vm.close()


def test_device_batch_layout_matches_host_batch():
    """bench.device_batch lays fixed-size batches out on the device (C4: 25 GB of UMEM); the bytes and
    descriptors must be workloads.build_batch's (checked here on a CPU tensor)."""
    import torch
    from gobpfld_amd import workloads as W
    B = _bench()
    for name in ("c4", "c2", "c3"):
        d_umem, d_desc, descs = B.device_batch(name, 77, 1000, torch.device("cpu"))
        umem, descs2 = W.build_batch(name, 77, 1000)
        assert np.array_equal(d_umem.numpy(), umem), name
        assert np.array_equal(descs, descs2), name
        assert np.array_equal(d_desc.numpy(), descs2.view(np.uint8)), name
