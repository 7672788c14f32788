"""GPU half of the shard exchange on one MI355X: two VMs on cuda:0 run the two shards
through xe_run_batch_multi (device delta kernels -> device sum -> apply, or the in-order replay with
device state export/import) and must equal the oracle's single VM over the whole batch: verdicts and
final maps, bit for bit. Covers the commuting configs, the u32-wrap program, two add widths on one
map, a cross-shard read of a counter an earlier shard adds to, and a non-atomic read-modify-write."""
import numpy as np
import pytest

from test_multirank import CASES, _batch, _dump, _oracle, _setup

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name,n,cap,commutes", CASES, ids=[c[0] for c in CASES])
def test_two_shards_on_one_gpu_equal_single_vm(gpu_lib, oracle_lib, name, n, cap, commutes):
    import torch
    from gobpfld_amd.emulator import Multi, VM, Settings
    G = 2
    vms = [VM(Settings(device=0), lib=gpu_lib) for _ in range(G)]
    for v in vms:
        _setup(v, name, cap)
    mu = Multi(vms)
    shard = n // G
    _batch.total = n
    host = [_batch(name, k * shard, shard) for k in range(G)]
    dev = [(torch.from_numpy(u).cuda(), torch.from_numpy(d.view(np.uint8)).cuda(),
            torch.zeros(shard, dtype=torch.int32, device="cuda")) for u, d in host]
    reps = []
    for step in range(2):
        _, rep = mu.run([u.data_ptr() for u, _, _ in dev], [u.numel() for u, _, _ in dev],
                        [d.data_ptr() for _, d, _ in dev], [shard] * G, d_verdicts=[v.data_ptr() for _, _, v in dev])
        reps.append(rep)
    torch.cuda.synchronize()
    r2, dumps = _oracle(oracle_lib, name, n, cap)
    ver = np.concatenate([v.cpu().numpy().view(np.uint32) for _, _, v in dev])
    assert (ver == r2.verdicts).all(), name
    for m, want in dumps.items():
        for k, v in enumerate(vms):
            assert _dump(v, m) == want, f"{name}: vm {k} map {m}"
    assert reps == [not commutes] * 2
    mu.close()
    for v in vms:
        v.close()
