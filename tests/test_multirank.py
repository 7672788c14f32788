"""N>1 path on CPU. world_size-2 `gloo` ranks each run a contiguous packet shard through the product's
device logic (host-simulation build) on private map replicas and then make their maps exact with
gobpfld_amd.shard.exchange_shards: a delta all-reduce when xe_shard_check proves the
shards' effects commute, the in-order replay otherwise. Every rank must end with the maps — and the
concatenated verdicts must equal the results — of the oracle's single VM over the whole batch.
The single-process form (xe_run_batch_multi, two VMs in one process) is checked the same way."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from gobpfld_amd import workloads as W

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CASES = [("c2", 8192, None, True), ("c5", 8192, 4096, True), ("u32wrap", 64, None, True),
         ("mixedwrap", 64, None, False), ("readvsadd", 256, None, False), ("addvsread", 256, None, True),
         ("rmw", 256, None, False), ("lru", 512, None, False), ("queue", 512, None, False)]
# shard epochs (several batches per exchange): a read of a field any other rank adds to needs the
# replay, so addvsread (rank 0 reads what rank 1 adds) no longer commutes
EPOCH_CASES = [c if c[0] != "addvsread" else (c[0], c[1], c[2], False) for c in CASES]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _batch(name, start, n):
    if name in ("readvsadd", "addvsread", "rmw"):
        # packets [0, n/2): byte 0 = 0 (adders); [n/2, n): byte 0 = 255 (readers) — addvsread: reversed
        from gobpfld_amd._native import np_dtypes
        d_desc, _, _ = np_dtypes()
        umem = np.zeros(n * 64, dtype=np.uint8)
        descs = np.zeros(n, dtype=d_desc)
        descs["addr"] = np.arange(n) * 64
        descs["len"] = 64
        second = np.arange(start, start + n) >= _batch.total // 2
        umem[::64] = np.where(second != (name == "addvsread"), 255, 0)
        return umem, descs
    return W.build_batch("c2" if name in ("u32wrap", "mixedwrap", "lru", "queue") else name, start, n)


_batch.total = 256


def _rank(rank, world, port, name, n, cap, out_dir):
    import sys
    sys.path.insert(0, ROOT)
    from gobpfld_amd import _native as N
    from gobpfld_amd.emulator import VM, Settings
    from gobpfld_amd.shard import exchange_shards
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lib = N.Lib(os.path.join(ROOT, "tests", "hostsim", "libxdpemu_hostsim.so"), "xe_")
    vm = VM(Settings(), lib=lib)
    _setup(vm, name, cap)
    shard = n // world
    _batch.total = n
    umem, descs = _batch(name, rank * shard, shard)
    ver = np.zeros(shard, dtype=np.uint32)
    run = lambda: vm.run_batch_device(umem.ctypes.data, umem.size, descs.ctypes.data, shard, d_verdicts=ver.ctypes.data)
    exact = []
    for step in range(2):  # two steps: each run's deltas / replay are against that run's start state
        run()
        exact.append(exchange_shards(vm, list(vm.map_defs), dist, run)["exact_sum"])
    np.save(os.path.join(out_dir, f"ver{rank}.npy"), ver)
    np.save(os.path.join(out_dir, f"exact{rank}.npy"), np.array(exact))
    for m in vm.map_defs:
        with open(os.path.join(out_dir, f"map{m}_r{rank}.bin"), "wb") as f:
            f.write(_dump(vm, m))
    vm.close()
    dist.destroy_process_group()


def _dump(vm, m):
    from gobpfld_amd.emulator import MAP_LRU_HASH
    d = vm.map_dump(m)
    if isinstance(d, bytes):
        return d
    if isinstance(d, list):  # QUEUE / STACK / PERF records in list order
        return b"|".join(d) + b"#" + str(len(d)).encode()
    keys, vals = d
    out = np.asarray(keys).tobytes() + b"|" + np.asarray(vals).tobytes()
    if vm.map_defs[m].type == MAP_LRU_HASH:
        out += b"|" + b"".join(vm.map_lru_order(m))
    return out


def _ordered_program(queue: bool):
    """Ordered maps (order-dependent by nature, so the shards always replay in order through the
    whole-state exchange of ordered maps). lru: LRU_HASH(4 entries) keyed by byte 0 & 7 — a hit returns
    the stored byte, a miss inserts byte 1 (evicting the least recently used key). queue: push byte 0
    onto a QUEUE (bpf_map_push_elem) and return byte 0."""
    from gobpfld_amd.asm import JEQ, Asm
    a = Asm()
    a.ldx(4, 6, 1, 0).ldx(1, 8, 6, 0)
    if queue:
        a.stx(8, 10, -8, 8).ld_map(1, 1).mov64(2, src=10).add64(2, -8).mov64(3, 0).call(87)
        a.mov64(0, src=8).exit()
        return a.assemble()
    a.alu64(0x50, 8, 7).stx(4, 10, -4, 8).ldx(1, 9, 6, 1).stx(8, 10, -16, 9)
    a.ld_map(1, 1).mov64(2, src=10).add64(2, -4).call(1)
    a.jmp(JEQ, 0, "miss", imm=0)
    a.ldx(8, 0, 0, 0).exit()
    a.label("miss")
    a.ld_map(1, 1).mov64(2, src=10).add64(2, -4).mov64(3, src=10).add64(3, -16).mov64(4, 0).call(2)
    a.mov64(0, 2).exit()
    return a.assemble()


def _wrap_program(mixed: bool):
    """u32 counter (low half of a u64 value) starting at 0xFFFFFFF0 wraps within its 4-byte field;
    `mixed` also adds to a u16 counter at offset 4 of the same value (two add widths on one map)."""
    from gobpfld_amd.asm import JEQ, Asm
    a = Asm()
    a.st(4, 10, -4, 0).ld_map(1, 1).mov64(2, src=10).add64(2, -4).call(1)
    a.jmp(JEQ, 0, "out", imm=0)
    a.mov64(1, 1).xadd(4, 0, 0, 1)
    if mixed:
        a.mov64(1, 0x4000).xadd(2, 0, 4, 1)
    a.label("out").mov64(0, 2).exit()
    return a.assemble()


def _role_program(rmw: bool):
    """Packets whose byte 0 is < 128 add 1 to a u64 counter; the others return its value (readvsadd),
    or (rmw) load, add and store it non-atomically — an ordered read-modify-write."""
    from gobpfld_amd.asm import JEQ, JGT, Asm
    a = Asm()
    a.ldx(4, 6, 1, 0).ldx(1, 8, 6, 0)
    a.st(4, 10, -4, 0).ld_map(1, 1).mov64(2, src=10).add64(2, -4).call(1)
    a.jmp(JEQ, 0, "out", imm=0)
    a.jmp(JGT, 8, "read", imm=127)
    a.mov64(1, 1).xadd(8, 0, 0, 1).mov64(0, 2).exit()
    a.label("read")
    if rmw:
        a.ldx(8, 1, 0, 0).add64(1, 3).stx(8, 0, 0, 1).mov64(0, src=1).exit()
    else:
        a.ldx(8, 0, 0, 0).exit()
    a.label("out").mov64(0, 1).exit()
    return a.assemble()


def _setup(vm, name, cap):
    from gobpfld_amd.emulator import MAP_ARRAY, MAP_LRU_HASH, MAP_QUEUE, MapDef
    if name in ("lru", "queue"):
        vm.add_map(MapDef(MAP_QUEUE, 0, 8, 1 << 16) if name == "queue" else MapDef(MAP_LRU_HASH, 4, 8, 4))
        vm.set_entrypoint(vm.add_raw_program(_ordered_program(name == "queue")))
        return
    if name in ("u32wrap", "mixedwrap"):
        vm.add_map(MapDef(MAP_ARRAY, 4, 8, 4), {0: (0xFFF0FFFFFFF0).to_bytes(8, "little")})
        vm.set_entrypoint(vm.add_raw_program(_wrap_program(name == "mixedwrap")))
        return
    if name in ("readvsadd", "addvsread", "rmw"):
        vm.add_map(MapDef(MAP_ARRAY, 4, 8, 1))
        vm.set_entrypoint(vm.add_raw_program(_role_program(name == "rmw")))
        return
    for mdef, ents in W.workload_maps(name):
        mi = vm.add_map(mdef)
        if ents is not None:
            keys, vals = ents
            vm.map_update_batch(mi, keys[:cap], vals[:cap])
    p = vm.add_raw_program(W.CONFIGS[name]["program"]())
    vm.set_entrypoint(p)


def _oracle(oracle_lib, name, n, cap, steps=2, all_results=False):
    """Single VM over the whole batch, `steps` times (the ranks run that many steps)."""
    from gobpfld_amd.emulator import VM, Settings
    ov = VM(Settings(), lib=oracle_lib)
    _setup(ov, name, cap)
    _batch.total = n
    umem, descs = _batch(name, 0, n)
    rs = [ov.run_batch(umem.copy(), descs) for _ in range(steps)]
    dumps = {m: _dump(ov, m) for m in ov.map_defs}
    ov.close()
    return (rs if all_results else rs[-1]), dumps


@pytest.mark.parametrize("name,n,cap,commutes", CASES, ids=[c[0] for c in CASES])
def test_two_rank_shards_equal_single_vm(tmp_path, oracle_lib, built, name, n, cap, commutes):
    world = 2
    mp.start_processes(_rank, args=(world, _free_port(), name, n, cap, str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    r2, dumps = _oracle(oracle_lib, name, n, cap)
    ver = np.concatenate([np.load(tmp_path / f"ver{r}.npy") for r in range(world)])
    assert (ver == r2.verdicts).all(), f"{name}: verdicts differ from the single VM"
    for m, want in dumps.items():
        for r in range(world):
            assert (tmp_path / f"map{m}_r{r}.bin").read_bytes() == want, f"rank {r} map {m}"
    exact = np.load(tmp_path / "exact0.npy")
    assert exact.all() == commutes and exact.any() == commutes, (name, exact)


@pytest.mark.parametrize("name,n,cap,commutes", CASES, ids=[c[0] for c in CASES])
def test_single_process_multi_equals_single_vm(oracle_lib, hostsim_lib, name, n, cap, commutes):
    """xe_run_batch_multi with two VMs in one process (host simulation: both on 'device' 0, so the
    exchange takes the device-kernel path instead of RCCL)."""
    from gobpfld_amd.emulator import Multi, VM, Settings
    G = 2
    vms = [VM(Settings(), lib=hostsim_lib) for _ in range(G)]
    for v in vms:
        _setup(v, name, cap)
    mu = Multi(vms)
    shard = n // G
    _batch.total = n
    bufs = [_batch(name, k * shard, shard) for k in range(G)]
    vers = [np.zeros(shard, dtype=np.uint32) for _ in range(G)]
    reps = []
    for step in range(2):
        _, rep = mu.run([u.ctypes.data for u, _ in bufs], [u.size for u, _ in bufs], [d.ctypes.data for _, d in bufs],
                        [shard] * G, d_verdicts=[v.ctypes.data for v in vers])
        reps.append(rep)
    r2, dumps = _oracle(oracle_lib, name, n, cap)
    assert (np.concatenate(vers) == r2.verdicts).all()
    for m, want in dumps.items():
        for k, v in enumerate(vms):
            assert _dump(v, m) == want, f"vm {k} map {m}"
    assert reps == [not commutes] * 2
    mu.close()
    for v in vms:
        v.close()


def _rank_epoch(rank, world, port, name, n, cap, out_dir, steps):
    import sys
    sys.path.insert(0, ROOT)
    from gobpfld_amd import _native as N
    from gobpfld_amd.emulator import VM, Settings
    from gobpfld_amd.shard import ShardEpoch
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lib = N.Lib(os.path.join(ROOT, "tests", "hostsim", "libxdpemu_hostsim.so"), "xe_")
    vm = VM(Settings(), lib=lib)
    _setup(vm, name, cap)
    shard = n // world
    _batch.total = n
    umem, descs = _batch(name, rank * shard, shard)
    pk = umem.copy()
    vers = [np.zeros(shard, dtype=np.uint32) for _ in range(steps)]

    def run(s, use_async=False):
        pk[:] = umem
        f = vm.run_batch_device_async if use_async else vm.run_batch_device
        return f(pk.ctypes.data, pk.size, descs.ctypes.data, shard, d_verdicts=vers[s].ctypes.data)

    ep = ShardEpoch(vm, list(vm.map_defs), dist)
    ep.begin()
    for s in range(steps):  # pipelined and synchronous batches in one epoch
        run(s, use_async=s % 2 == 0)
    vm.sync()
    x = ep.exchange([lambda s=s: run(s) for s in range(steps)])
    np.save(os.path.join(out_dir, f"ver{rank}.npy"), np.stack(vers))
    np.save(os.path.join(out_dir, f"exact{rank}.npy"), np.array([x["exact_sum"]]))
    for m in vm.map_defs:
        with open(os.path.join(out_dir, f"map{m}_r{rank}.bin"), "wb") as f:
            f.write(_dump(vm, m))
    vm.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("name,n,cap,commutes", EPOCH_CASES, ids=[c[0] for c in EPOCH_CASES])
def test_two_rank_epoch_equals_single_vm(tmp_path, oracle_lib, built, name, n, cap, commutes):
    """Three batches per rank in one shard epoch, one exchange: every batch's verdicts and the final
    maps equal the oracle's single VM walking the three whole batches in order."""
    world, steps = 2, 3
    mp.start_processes(_rank_epoch, args=(world, _free_port(), name, n, cap, str(tmp_path), steps), nprocs=world,
                       join=True, start_method="spawn")
    rs, dumps = _oracle(oracle_lib, name, n, cap, steps=steps, all_results=True)
    ver = np.concatenate([np.load(tmp_path / f"ver{r}.npy") for r in range(world)], axis=1)
    for s in range(steps):
        assert (ver[s] == rs[s].verdicts).all(), f"{name}: batch {s} verdicts differ from the single VM"
    for m, want in dumps.items():
        for r in range(world):
            assert (tmp_path / f"map{m}_r{r}.bin").read_bytes() == want, f"rank {r} map {m}"
    assert bool(np.load(tmp_path / "exact0.npy")[0]) == commutes


def _rank_bench(rank, world, port, name, n, out_dir):
    """bench.run_epochs itself (warm-up epoch + timed epoch, pipelined batches, the shard exchange inside
    the timed region) on host-simulation VMs over CPU tensors."""
    import importlib.util
    import sys
    sys.path.insert(0, ROOT)
    from gobpfld_amd import _native as N
    from gobpfld_amd.emulator import VM, Settings
    from gobpfld_amd.shard import ShardEpoch
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    B = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(B)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lib = N.Lib(os.path.join(ROOT, "tests", "hostsim", "libxdpemu_hostsim.so"), "xe_")
    vm = VM(Settings(), lib=lib)
    _setup(vm, name, None)
    shard = n // world
    _batch.total = n
    umem, descs = _batch(name, rank * shard, shard)
    dev = torch.device("cpu")
    d_umem = torch.from_numpy(umem.copy())
    d_desc = torch.from_numpy(descs.view(np.uint8).copy())
    d_ver = torch.zeros(shard, dtype=torch.int32)
    epoch = ShardEpoch(vm, list(vm.map_defs), dist)
    sts, elapsed, x_s, exchanges = B.run_epochs(vm, epoch, dist, world, dev, d_umem, d_desc, shard, d_ver, None, 1, 2)
    np.save(os.path.join(out_dir, f"ver{rank}.npy"), d_ver.numpy().view(np.uint32))
    np.save(os.path.join(out_dir, f"x{rank}.npy"), np.array([exchanges["exact_sum"], exchanges["replayed"], len(sts)]))
    for m in vm.map_defs:
        with open(os.path.join(out_dir, f"map{m}_r{rank}.bin"), "wb") as f:
            f.write(_dump(vm, m))
    vm.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("name,n,replays", [("readvsadd", 256, True), ("c2", 8192, False)])
def test_bench_run_epochs_two_ranks(tmp_path, oracle_lib, built, name, n, replays):
    """The bench's own epoch loop at world size 2 (gloo): a read-vs-add program (rank 1's packets read the
    counter rank 0's packets add to) must take the exchange's in-order replay branch in both epochs, C2
    the exact delta sum; either way every rank ends with the oracle's single VM after 1 + 2 batches, and
    the last verdicts are that VM's last run."""
    world = 2
    mp.start_processes(_rank_bench, args=(world, _free_port(), name, n, str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    r3, dumps = _oracle(oracle_lib, name, n, None, steps=3)
    ver = np.concatenate([np.load(tmp_path / f"ver{r}.npy") for r in range(world)])
    assert (ver == r3.verdicts).all(), f"{name}: last verdicts differ from the single VM"
    for m, want in dumps.items():
        for r in range(world):
            assert (tmp_path / f"map{m}_r{r}.bin").read_bytes() == want, f"rank {r} map {m}"
    x = np.load(tmp_path / "x0.npy")
    assert x[2] == 2, "two timed batches"
    assert list(x[:2]) == ([0, 2] if replays else [2, 0]), x  # warm-up and timed epochs: replayed / exact sums
