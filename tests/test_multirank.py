"""N>1 path on CPU: world_size-2 `gloo` ranks each run a contiguous packet shard through the product
(host-simulation build) on private map replicas, exchange counter deltas with one all-reduce (the
bench's RCCL step), and must end with maps equal to the oracle's single VM over the whole
batch (valid because the configs' map effects are commutative)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from gobpfld_amd import workloads as W

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank(rank, world, port, name, n, cap, out_dir):
    import sys
    sys.path.insert(0, ROOT)
    from gobpfld_amd import _native as N
    from gobpfld_amd.emulator import VM, Settings
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lib = N.Lib(os.path.join(ROOT, "tests", "hostsim", "libxdpemu_hostsim.so"), "xe_")
    vm = VM(Settings(), lib=lib)
    _setup(vm, name, cap)
    shard = n // world
    umem, descs = W.build_batch("c2" if name == "u32wrap" else name, rank * shard, shard)
    ver = np.zeros(shard, dtype=np.uint32)
    from gobpfld_amd.shard import allreduce_map_deltas
    bufs = {m: torch.zeros(vm.map_values_bytes(m), dtype=torch.uint8) for m in vm.map_defs}
    for step in range(2):  # two steps: deltas are per batch, against that batch's snapshot
        vm.run_batch_device(umem.ctypes.data, umem.size, descs.ctypes.data, shard, d_verdicts=ver.ctypes.data)
        allreduce_map_deltas(vm, list(vm.map_defs), bufs, dist)
    np.save(os.path.join(out_dir, f"ver{rank}.npy"), ver)
    for m in vm.map_defs:
        with open(os.path.join(out_dir, f"map{m}_r{rank}.bin"), "wb") as f:
            f.write(_dump(vm, m))
    vm.close()
    dist.destroy_process_group()


def _dump(vm, m):
    d = vm.map_dump(m)
    if isinstance(d, bytes):
        return d
    keys, vals = d
    return np.asarray(keys).tobytes() + b"|" + np.asarray(vals).tobytes()


def _u32wrap_program():
    """u32 counter (low half of a u64 value) starting at 0xFFFFFFF0: wraps within its 4-byte field."""
    from gobpfld_amd.asm import JEQ, Asm
    a = Asm()
    a.st(4, 10, -4, 0).ld_map(1, 1).mov64(2, src=10).add64(2, -4).call(1)
    a.jmp(JEQ, 0, "out", imm=0)
    a.mov64(1, 1).xadd(4, 0, 0, 1)
    a.label("out").mov64(0, 2).exit()
    return a.assemble()


def _setup(vm, name, cap):
    if name == "u32wrap":
        from gobpfld_amd.emulator import MAP_ARRAY, MapDef
        vm.add_map(MapDef(MAP_ARRAY, 4, 8, 4), (0xFFFFFFF0).to_bytes(8, "little") + bytes(24))
        vm.set_entrypoint(vm.add_raw_program(_u32wrap_program()))
        return
    for mdef, ents in W.workload_maps(name):
        mi = vm.add_map(mdef)
        if ents is not None:
            keys, vals = ents
            vm.map_update_batch(mi, keys[:cap], vals[:cap])
    p = vm.add_raw_program(W.CONFIGS[name]["program"]())
    vm.set_entrypoint(p)


@pytest.mark.parametrize("name,n,cap", [("c2", 8192, None), ("c5", 8192, 4096), ("u32wrap", 64, None)])
def test_two_rank_shards_equal_single_vm(tmp_path, oracle_lib, built, name, n, cap):
    world = 2
    mp.start_processes(_rank, args=(world, _free_port(), name, n, cap, str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    from gobpfld_amd.emulator import VM, Settings
    ov = VM(Settings(), lib=oracle_lib)
    _setup(ov, name, cap)
    umem, descs = W.build_batch("c2" if name == "u32wrap" else name, 0, n)
    r1 = ov.run_batch(umem.copy(), descs)
    r2 = ov.run_batch(umem.copy(), descs)
    ver = np.concatenate([np.load(tmp_path / f"ver{r}.npy") for r in range(world)])
    assert (ver == r2.verdicts).all() and (r1.verdicts == r2.verdicts).all()
    for m in ov.map_defs:
        want = _dump(ov, m)
        for r in range(world):
            assert (tmp_path / f"map{m}_r{r}.bin").read_bytes() == want, f"rank {r} map {m}"
    ov.close()
