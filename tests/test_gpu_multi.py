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


EPOCH_GPU = [("c2", 8192, None), ("c5", 8192, 4096), ("u32wrap", 64, None)]


@pytest.mark.parametrize("name,n,cap", EPOCH_GPU, ids=[c[0] for c in EPOCH_GPU])
def test_epoch_two_shards_on_one_gpu(gpu_lib, oracle_lib, name, n, cap):
    """Shard epoch on the device: two VMs on cuda:0 each run three pipelined batches after
    xe_epoch_begin; xe_shard_check over the epoch footprints, xe_map_delta against the epoch's start,
    a device sum and xe_map_apply_delta then give both VMs the oracle's maps after the three whole
    batches, and every batch's verdicts equal the oracle's."""
    import torch
    from gobpfld_amd.emulator import VM, Settings
    G, steps = 2, 3
    vms = [VM(Settings(device=0), lib=gpu_lib) for _ in range(G)]
    for v in vms:
        _setup(v, name, cap)
    shard = n // G
    _batch.total = n
    host = [_batch(name, k * shard, shard) for k in range(G)]
    dev = [(torch.from_numpy(u).cuda(), torch.from_numpy(d.view(np.uint8)).cuda()) for u, d in host]
    vers = [[torch.zeros(shard, dtype=torch.int32, device="cuda") for _ in range(steps)] for _ in range(G)]
    for v in vms:
        v.epoch_begin()
    for s in range(steps):
        for k, v in enumerate(vms):
            u, d = dev[k]
            v.run_batch_device_async(u.data_ptr(), u.numel(), d.data_ptr(), shard, d_verdicts=vers[k][s].data_ptr())
    for v in vms:
        v.sync()
    fps = np.concatenate([v.footprint() for v in vms])
    ok, lanes = vms[0].shard_check(fps, G)
    assert ok, "commuting programs must pass the epoch check"
    for m in vms[0].map_defs:
        lane = lanes[m - 1]
        if not lane:
            continue
        nb = vms[0].map_values_bytes(m) * (2 if lane == 2 else 1)
        bufs = [torch.zeros(nb, dtype=torch.uint8, device="cuda") for _ in vms]
        for v, b in zip(vms, bufs):
            v.map_delta(m, b.data_ptr(), lane=lane)
        w = {1: torch.uint8, 2: torch.int32, 4: torch.int32, 8: torch.int64}[lane]
        tot = bufs[0].view(w) + bufs[1].view(w)
        torch.cuda.synchronize()  # the sum runs on torch's stream, the apply on each VM's
        for v in vms:
            v.map_apply_delta(m, tot.view(torch.uint8).data_ptr(), lane=lane)
    for v in vms:
        v.epoch_end()
    torch.cuda.synchronize()
    rs, dumps = _oracle(oracle_lib, name, n, cap, steps=steps, all_results=True)
    for s in range(steps):
        ver = np.concatenate([vers[k][s].cpu().numpy().view(np.uint32) for k in range(G)])
        assert (ver == rs[s].verdicts).all(), f"{name}: batch {s}"
    for m, want in dumps.items():
        for k, v in enumerate(vms):
            assert _dump(v, m) == want, f"{name}: vm {k} map {m}"
    for v in vms:
        v.close()


def test_shard_epoch_bench_path_one_rank(gpu_lib, oracle_lib):
    """The bench's N > 1 step path (ShardEpoch over torch.distributed with backend nccl = RCCL) at
    world size 1 on cuda:0: pipelined C2 batches in an epoch, the footprint all-gather, the check and
    the delta all-reduce leave the maps equal to the oracle's after the same batches."""
    import socket

    import torch
    import torch.distributed as dist

    from gobpfld_amd.emulator import VM, Settings
    from gobpfld_amd.shard import ShardEpoch
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        n, steps = 8192, 3
        vm = VM(Settings(device=0), lib=gpu_lib)
        _setup(vm, "c2", None)
        _batch.total = n
        u, d = _batch("c2", 0, n)
        du, dd = torch.from_numpy(u).cuda(), torch.from_numpy(d.view(np.uint8)).cuda()
        ver = torch.zeros(n, dtype=torch.int32, device="cuda")
        stream = torch.cuda.current_stream().cuda_stream
        run = lambda: vm.run_batch_device(du.data_ptr(), du.numel(), dd.data_ptr(), n, d_verdicts=ver.data_ptr(), stream=stream)
        ep = ShardEpoch(vm, list(vm.map_defs), dist, device=torch.device("cuda", 0), stream=stream)
        ep.begin()
        for _ in range(steps):
            vm.run_batch_device_async(du.data_ptr(), du.numel(), dd.data_ptr(), n, d_verdicts=ver.data_ptr(), stream=stream)
        vm.sync()
        x = ep.exchange([run] * steps)
        torch.cuda.synchronize()
        assert x["exact_sum"]
        rs, dumps = _oracle(oracle_lib, "c2", n, None, steps=steps, all_results=True)
        assert (ver.cpu().numpy().view(np.uint32) == rs[-1].verdicts).all()
        for m, want in dumps.items():
            assert _dump(vm, m) == want
        vm.close()
    finally:
        dist.destroy_process_group()


def _gloo_rank(rank, world, port, name, n, k, out):
    """One rank of the bench's N > 1 path (ShardEpoch over torch.distributed) sharing cuda:0 with the
    other over gloo: pipelined batches, the exchange, then the map against the header truth."""
    import importlib.util
    import os

    import torch
    import torch.distributed as dist

    from gobpfld_amd import workloads as W
    from gobpfld_amd.emulator import VM, Settings
    from gobpfld_amd.shard import ShardEpoch
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(root, "bench.py"))
    B = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(B)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    vm = VM(Settings())
    W.setup_vm(vm, name)
    umem, descs = W.build_batch(name, rank * n, n)
    du, dd = torch.from_numpy(umem).to(dev), torch.from_numpy(descs.view(np.uint8)).to(dev)
    ver = torch.zeros(n, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream(dev).cuda_stream  # 0 on the default stream: the library uses its own
    ep = ShardEpoch(vm, list(vm.map_defs), dist, device=dev, stream=stream)
    run = lambda: vm.run_batch_device(du.data_ptr(), du.numel(), dd.data_ptr(), n, d_verdicts=ver.data_ptr(), stream=stream)
    exact = []
    for _ in range(2):  # two epochs of k pipelined batches
        ep.begin()
        for _ in range(k):
            vm.run_batch_device_async(du.data_ptr(), du.numel(), dd.data_ptr(), n, d_verdicts=ver.data_ptr(), stream=stream)
        vm.sync()
        exact.append(ep.exchange([run] * k)["exact_sum"])
    r = B.verify(name, vm, rank * n, n, 2 * k, ver, dist, world, dev)
    np.save(os.path.join(out, f"r{rank}.npy"), np.array([r["verified"], r["map_ok_rank0"], all(exact)]))
    vm.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("name", ["c5", "c3", "c2"])
def test_shard_epoch_two_ranks_share_one_gpu(tmp_path, name):
    """bench.py's N > 1 exchange with two processes on cuda:0 (gloo): after two epochs every rank's map
    is init + 4 runs x (shard 0 + shard 1) of the header truth. Catches the library reading a delta
    buffer before the collective that fills it has landed (stream 0 is not torch's default stream)."""
    import socket

    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.spawn(_gloo_rank, args=(2, port, name, 1 << 18, 2, str(tmp_path)), nprocs=2)
    for r in range(2):
        verified, map_ok, exact = np.load(tmp_path / f"r{r}.npy", allow_pickle=False)
        assert exact and map_ok and verified, f"{name}: rank {r}: exact {exact} map {map_ok} verified {verified}"
