"""Pipelined batches (xe_run_batch_device_async / xe_sync): a stream of batches queued without waiting
must give exactly what the reference harness gives when it walks the same packets batch after batch
(SURVEY Appendix B): per-packet verdicts and the final maps equal the oracle's single VM run over the
batches in order. A batch whose conflict check asks for the in-order replay must stop the batches
queued behind it and be replayed with them, still in submission order.

CPU: the host simulation build (device pointers are host pointers). GPU (-m gpu): the product on
cuda:0, including the full-size C2 stream."""
import numpy as np
import pytest

from gobpfld_amd import workloads as W
from gobpfld_amd.asm import JNE, Asm
from gobpfld_amd.emulator import MAP_ARRAY, MODE_KEYED, MODE_PARALLEL, MODE_SEQUENTIAL, VM, MapDef, Settings
from parity import packets

MARK = 0xEE


def prog_mixed():
    """key = byte 0 & 7 into ARRAY(8 x 16 B); byte 1 == MARK: a plain store of byte 2 into value[0..8)
    (an order-dependent write: the batch replays in order); otherwise an atomic add of 1 at value[8]."""
    a = Asm()
    a.ldx(4, 6, 1, 0)
    a.ldx(1, 8, 6, 0).alu64(0x50, 8, 7)      # r8 = byte 0 & 7
    a.ldx(1, 9, 6, 1)                        # r9 = byte 1
    a.ldx(1, 7, 6, 2)                        # r7 = byte 2
    a.stx(4, 10, -4, 8).ld_map(1, 1).mov64(2, src=10).add64(2, -4).call(1)
    a.jmp(0x15, 0, "out", imm=0)             # JEQ r0, 0
    a.jmp(JNE, 9, "add", imm=MARK)
    a.stx(8, 0, 0, 7)                        # value[0..8) = byte 2
    a.ja("out")
    a.label("add").mov64(1, 1).xadd(8, 0, 8, 1)
    a.label("out").mov64(0, 2).exit()
    return a.assemble()


def batches(n_batches: int, n: int, marked: set[int]):
    """Packets per batch; batch b in `marked` carries a few MARK packets (the rest never do)."""
    out = []
    for b in range(n_batches):
        umem, descs = packets(n, 64, seed=100 + b)
        pk = umem.reshape(n, 64)
        pk[pk[:, 1] == MARK, 1] = 0
        if b in marked:
            pk[[3, n // 2, n - 5], 1] = MARK
        out.append((umem, descs))
    return out


def oracle_stream(oracle_lib, prog, bs, entries=8):
    vm = VM(Settings(), lib=oracle_lib)
    m = vm.add_map(MapDef(MAP_ARRAY, 4, 16, entries))
    vm.set_entrypoint(vm.add_raw_program(prog))
    ver = [vm.run_batch(u.copy(), d, want_regs=False).verdicts for u, d in bs]
    dump = vm.map_dump(m)
    vm.close()
    return ver, dump


def host_stream(lib, prog, bs, use_async: bool, mode=0, entries=8):
    """Run the batches through the device-resident entry points of the host simulation (host memory)."""
    vm = VM(Settings(mode=mode), lib=lib)
    m = vm.add_map(MapDef(MAP_ARRAY, 4, 16, entries))
    vm.set_entrypoint(vm.add_raw_program(prog))
    keep, handles = [], []
    for u, d in bs:
        u = u.copy()
        v = np.zeros(len(d), dtype=np.uint32)
        keep.append((u, d, v))
        run = vm.run_batch_device_async if use_async else vm.run_batch_device
        handles.append(run(u.ctypes.data, u.nbytes, d.ctypes.data, len(d), d_verdicts=v.ctypes.data))
    sts = [h.stats() for h in handles] if use_async else handles
    dump = vm.map_dump(m)
    vm.close()
    return [k[2] for k in keep], sts, dump


# 8 entries: a small value region (the kernel's batch tail folds and snapshots it); 4096: a large one
# (the prologue snapshot and the replica fold launch)
@pytest.mark.parametrize("entries", [8, 4096])
@pytest.mark.parametrize("marked", [set(), {2}, {0, 3}, {5}], ids=["clean", "middle", "first_and_later", "last"])
def test_async_stream_equals_oracle_hostsim(hostsim_lib, oracle_lib, marked, entries):
    prog = prog_mixed()
    bs = batches(6, 512, marked)
    ver_o, dump_o = oracle_stream(oracle_lib, prog, bs, entries)
    ver_a, st_a, dump_a = host_stream(hostsim_lib, prog, bs, True, entries=entries)
    ver_s, st_s, dump_s = host_stream(hostsim_lib, prog, bs, False, entries=entries)
    assert dump_a == dump_o == dump_s
    for b in range(len(bs)):
        assert (ver_a[b] == ver_o[b]).all() and (ver_s[b] == ver_o[b]).all(), f"batch {b}"
        want_seq = b in marked
        # the marked store writes one map entry: keyed ordered execution (its key's chain in order)
        assert st_a[b]["mode_used"] == (MODE_KEYED if want_seq else MODE_PARALLEL), (b, st_a[b])
        assert st_a[b]["conflict"] == int(want_seq)
        assert st_a[b]["status_count"] == st_s[b]["status_count"] and st_a[b]["steps"] == st_s[b]["steps"]


def test_async_map_access_completes_pipeline(hostsim_lib):
    """A map read between pipelined batches sees every batch queued before it."""
    prog = prog_mixed()
    bs = batches(3, 256, set())
    vm = VM(Settings(), lib=hostsim_lib)
    m = vm.add_map(MapDef(MAP_ARRAY, 4, 16, 8))
    vm.set_entrypoint(vm.add_raw_program(prog))
    keep = []
    for u, d in bs:
        u = u.copy()
        keep.append(u)
        vm.run_batch_device_async(u.ctypes.data, u.nbytes, d.ctypes.data, len(d))
    raw = np.frombuffer(vm.map_dump(m), dtype=np.uint64).reshape(8, 2)
    assert int(raw[:, 1].sum()) == 3 * 256  # every packet added 1
    vm.close()


def host_update_between(lib, prog, bs, kind, entries):
    """Batches with a host map update between them (the staged snapshot must not outlive it); kind:
    "oracle" (run_batch on the oracle), "sync" or "async" (device entry points on host memory)."""
    vm = VM(Settings(), lib=lib)
    m = vm.add_map(MapDef(MAP_ARRAY, 4, 16, entries))
    vm.set_entrypoint(vm.add_raw_program(prog))
    for b, (u, d) in enumerate(bs):
        u = u.copy()
        if kind == "async":
            vm.run_batch_device_async(u.ctypes.data, u.nbytes, d.ctypes.data, len(d))
        elif kind == "oracle":
            vm.run_batch(u, d, want_regs=False)
        else:
            vm.run_batch_device(u.ctypes.data, u.nbytes, d.ctypes.data, len(d))
        if b == 1:
            vm.map_update(m, np.uint32(3).tobytes(), np.arange(16, dtype=np.uint8).tobytes())
    dump = vm.map_dump(m)
    vm.close()
    return dump


@pytest.mark.parametrize("entries", [8, 4096])
def test_async_host_update_between_batches(hostsim_lib, oracle_lib, entries):
    """A host map update between pipelined batches reaches the later batches and their rollback points:
    a replayed batch after the update starts from the updated value."""
    prog = prog_mixed()
    bs = batches(4, 256, {3})
    want = host_update_between(oracle_lib, prog, bs, "oracle", entries)
    assert host_update_between(hostsim_lib, prog, bs, "sync", entries) == want
    assert host_update_between(hostsim_lib, prog, bs, "async", entries) == want


def test_async_delta_needs_sync_batch(hostsim_lib):
    """Shard deltas are taken against a synchronous batch's start: refused after pipelined batches."""
    from gobpfld_amd.emulator import EmulatorError
    prog = prog_mixed()
    (u, d), = batches(1, 128, set())
    vm = VM(Settings(), lib=hostsim_lib)
    m = vm.add_map(MapDef(MAP_ARRAY, 4, 16, 8))
    vm.set_entrypoint(vm.add_raw_program(prog))
    u = u.copy()
    vm.run_batch_device_async(u.ctypes.data, u.nbytes, d.ctypes.data, len(d)).stats()
    out = np.zeros(128, dtype=np.uint8)
    with pytest.raises(EmulatorError):
        vm.map_delta(m, out.ctypes.data)
    vm.run_batch_device(u.ctypes.data, u.nbytes, d.ctypes.data, len(d))
    vm.map_delta(m, out.ctypes.data)
    vm.close()


# ------------------------------------------------------------------------------------------ GPU
@pytest.mark.gpu
@pytest.mark.parametrize("entries", [8, 4096])
@pytest.mark.parametrize("marked", [set(), {2}, {0, 3}], ids=["clean", "middle", "first_and_later"])
def test_async_stream_equals_oracle_gpu(gpu_lib, oracle_lib, marked, entries):
    import torch
    prog = prog_mixed()
    bs = batches(6, 4096, marked)
    ver_o, dump_o = oracle_stream(oracle_lib, prog, bs, entries)
    vm = VM(Settings(), lib=gpu_lib)
    m = vm.add_map(MapDef(MAP_ARRAY, 4, 16, entries))
    vm.set_entrypoint(vm.add_raw_program(prog))
    dev, hs = [], []
    for u, d in bs:
        du = torch.from_numpy(u).cuda()
        dd = torch.from_numpy(d.view(np.uint8)).cuda()
        dv = torch.zeros(len(d), dtype=torch.int32, device="cuda")
        dev.append((du, dd, dv))
        hs.append(vm.run_batch_device_async(du.data_ptr(), du.numel(), dd.data_ptr(), len(d), d_verdicts=dv.data_ptr()))
    sts = [h.stats() for h in hs]
    assert vm.map_dump(m) == dump_o
    for b, (_, _, dv) in enumerate(dev):
        assert (dv.cpu().numpy().view(np.uint32) == ver_o[b]).all(), f"batch {b}"
        assert sts[b]["mode_used"] == (MODE_KEYED if b in marked else MODE_PARALLEL), (b, sts[b])
    vm.close()


@pytest.mark.gpu
def test_async_c2_full_size_stream(gpu_lib):
    """Five pipelined 16M-packet C2 batches: verdicts and counters equal five synchronous batches."""
    import torch
    n = 16 * 1024 * 1024
    umem, descs = W.build_batch("c2", 0, n)
    d_umem = torch.from_numpy(umem).cuda()
    d_desc = torch.from_numpy(descs.view(np.uint8)).cuda()
    out = {}
    for use_async in (False, True):
        vm = VM(Settings(), lib=gpu_lib)
        W.setup_vm(vm, "c2")
        d_ver = torch.zeros(n, dtype=torch.int32, device="cuda")
        run = vm.run_batch_device_async if use_async else vm.run_batch_device
        hs = [run(d_umem.data_ptr(), d_umem.numel(), d_desc.data_ptr(), n, d_verdicts=d_ver.data_ptr()) for _ in range(5)]
        sts = [h.stats() for h in hs] if use_async else hs
        torch.cuda.synchronize()
        out[use_async] = (vm.map_dump(1), d_ver.cpu().numpy(), [s["status_count"] for s in sts], [s["steps"] for s in sts])
        assert all(s["mode_used"] == MODE_PARALLEL and s["conflict"] == 0 for s in sts)
        vm.close()
    assert out[True][0] == out[False][0]
    assert (out[True][1] == out[False][1]).all()
    assert out[True][2] == out[False][2] and out[True][3] == out[False][3]


@pytest.mark.gpu
@pytest.mark.parametrize("entries", [8, 4096])
def test_async_host_update_between_batches_gpu(gpu_lib, oracle_lib, entries):
    """On the device: a host map update between pipelined batches reaches the later batches and the
    rollback point of a replayed one."""
    import torch
    prog = prog_mixed()
    bs = batches(4, 4096, {3})
    want = host_update_between(oracle_lib, prog, bs, "oracle", entries)
    vm = VM(Settings(), lib=gpu_lib)
    m = vm.add_map(MapDef(MAP_ARRAY, 4, 16, entries))
    vm.set_entrypoint(vm.add_raw_program(prog))
    keep = []
    for b, (u, d) in enumerate(bs):
        du = torch.from_numpy(u).cuda()
        dd = torch.from_numpy(d.view(np.uint8)).cuda()
        keep.append((du, dd))
        vm.run_batch_device_async(du.data_ptr(), du.numel(), dd.data_ptr(), len(d))
        if b == 1:
            vm.map_update(m, np.uint32(3).tobytes(), np.arange(16, dtype=np.uint8).tobytes())
    assert vm.map_dump(m) == want
    vm.close()


@pytest.mark.gpu
def test_async_c5_stream(gpu_lib):
    """Pipelined C5 batches (a 1M-flow HASH map: prologue snapshot, no tail fold; paired adds): the
    counters equal those of the same batches run synchronously."""
    import torch
    n = 1 << 20
    umem, descs = W.build_batch("c5", 0, n)
    d_umem = torch.from_numpy(umem).cuda()
    d_desc = torch.from_numpy(descs.view(np.uint8)).cuda()
    out = {}
    for use_async in (False, True):
        vm = VM(Settings(), lib=gpu_lib)
        W.setup_vm(vm, "c5")
        d_ver = torch.zeros(n, dtype=torch.int32, device="cuda")
        run = vm.run_batch_device_async if use_async else vm.run_batch_device
        hs = [run(d_umem.data_ptr(), d_umem.numel(), d_desc.data_ptr(), n, d_verdicts=d_ver.data_ptr()) for _ in range(4)]
        sts = [h.stats() for h in hs] if use_async else hs
        torch.cuda.synchronize()
        keys, vals = vm.map_dump(1)
        out[use_async] = (keys, vals, d_ver.cpu().numpy(), [s["status_count"] for s in sts])
        assert all(s["mode_used"] == MODE_PARALLEL and s["conflict"] == 0 for s in sts)
        vm.close()
    for k in range(3):
        assert np.array_equal(out[True][k], out[False][k])
    assert out[True][3] == out[False][3]
    assert int(out[True][1].view(np.uint64).reshape(-1, 2)[:, 0].sum()) > 0
