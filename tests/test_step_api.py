"""The batch counterparts of the reference VM's step-level API (VERDICT r3 "missing" 3 and 4):

  * the instruction trace (xe_trace_config / xe_trace_read): after every Step that returns without an
    error, the registers VM.String prints (emulator/vm.go:137-173, 248-270), for selected packets;
  * the replaceable helper table (VM.HelperFunctions, emulator/vm.go:23,35; HelperFunc,
    emulator/helper_functions.go:17): host functions and nil entries (inst_call_helper.go:20-36);
  * cancellation of pipelined batches (RunContext's ctx.Err(), emulator/vm.go:117-134): xe_cancel.

Parity: the oracle records its own Steps (oracle/oracle.cpp orc_trace_*) and calls host functions from its
per-packet loop; the implementation under test (host simulation on CPU, the product on the GPU) must give
the same records, the same calls in the same (packet) order and the same results. The reference holds no
step traces, so the trace comparison is "parity unpinned" beyond the oracle's reading of vm.go."""
import numpy as np
import pytest

from gobpfld_amd import workloads as W
from gobpfld_amd.asm import Asm
from gobpfld_amd.emulator import (ENGINE_INTERP, MAP_ARRAY, MODE_CANCELLED, MODE_PARALLEL, MODE_SEQUENTIAL, VM,
                                  E_HOST_HELPER, E_IN_HELPER, EmulatorError, MapDef, Settings)
from fuzz import gen_program
from kats import KATS
from parity import assert_same, packets, setup_one

FRAMEPTR, MEMPTR, IMM = 2, 1, 0


def _traced_run(lib, program, maps, entries, umem, descs, pk, max_steps, settings=None):
    vm, _ = setup_one(lib, program, maps, settings, entries)
    vm.trace(pk, max_steps)
    r = vm.run_batch(umem.copy(), descs, want_regs=True)
    tr = {p: vm.trace_read(p) for p in pk if p < len(descs)}
    vm.close()
    return r, tr


def _same_trace(a, b, what):
    assert a.keys() == b.keys()
    for p in a:
        ta, tb = a[p], b[p]
        assert len(ta) == len(tb), f"{what} packet {p}: {len(ta)} steps recorded, oracle {len(tb)}"
        if not len(ta):
            continue
        for f in ("packet", "step", "pc", "pi", "sf", "kind", "val"):
            bad = np.nonzero((ta[f] != tb[f]).reshape(len(ta), -1).any(axis=1))[0]
            assert not len(bad), f"{what} packet {p} step {bad[0]}: {f} {ta[bad[0]][f]} != oracle {tb[bad[0]][f]}"


# ------------------------------------------------------------------------------------------- trace
def test_trace_known_sequence(oracle_lib, hostsim_lib):
    """r0 = 1; r0 += 2; exit: three Steps, each recorded with the registers after it."""
    a = Asm()
    a.mov64(0, 1).alu64(0x00, 0, 2).exit()
    umem, descs = packets(2, 64)
    for lib in (oracle_lib, hostsim_lib):
        _, tr = _traced_run(lib, a.assemble(), [], None, umem, descs, [1], 16)
        t = tr[1]
        assert list(t["step"]) == [0, 1, 2] and list(t["pc"]) == [0, 1, 2]
        assert list(t["val"][:, 0]) == [1, 3, 3] and (t["kind"][:, 0] == IMM).all()
        assert (t["pi"] == 1).all() and (t["sf"] == 0).all() and (t["packet"] == 1).all()
        assert (t["kind"][:, 1] == MEMPTR).all() and (t["val"][:, 1] == 0).all()   # R1 = &ctx
        assert (t["kind"][:, 10] == FRAMEPTR).all() and (t["val"][:, 10] == 0).all()  # R10: frame 0, offset 0


@pytest.mark.parametrize("k", KATS, ids=[k["name"] for k in KATS])
def test_trace_kats_hostsim_equals_oracle(oracle_lib, hostsim_lib, k):
    umem, descs = packets(4, k["pkt"], seed=7)
    a = _traced_run(hostsim_lib, k["program"], k["maps"], k["entries"], umem, descs, [0, 3], 300)
    b = _traced_run(oracle_lib, k["program"], k["maps"], k["entries"], umem, descs, [0, 3], 300)
    _same_trace(a[1], b[1], k["name"])
    assert (a[0].results == b[0].results).all()


@pytest.mark.parametrize("seed", range(12))
def test_trace_fuzz_hostsim_equals_oracle(oracle_lib, hostsim_lib, seed):
    prog, maps, entries, settings = gen_program(seed, 24 + seed % 64)
    umem, descs = packets(64, 128, seed=seed)
    pk = [0, 5, 63]
    a = _traced_run(hostsim_lib, prog, maps, entries, umem, descs, pk, 2000, settings)
    b = _traced_run(oracle_lib, prog, maps, entries, umem, descs, pk, 2000, settings)
    _same_trace(a[1], b[1], f"fuzz {seed}")


def test_trace_truncates_and_rejects(oracle_lib, hostsim_lib):
    a = Asm()
    for _ in range(10):
        a.alu64(0x00, 0, 1)
    a.exit()
    umem, descs = packets(3, 64)
    for lib in (oracle_lib, hostsim_lib):
        vm, _ = setup_one(lib, a.assemble(), [])
        vm.trace([2, 2, 0], 4)  # duplicates collapse
        vm.run_batch(umem.copy(), descs)
        t = vm.trace_read(2)
        assert len(t) == 4 and list(t["val"][:, 0]) == [1, 2, 3, 4]
        with pytest.raises(EmulatorError):
            vm.trace_read(1)  # not traced
        vm.trace([])  # off
        vm.run_batch(umem.copy(), descs)
        vm.close()


def test_trace_follows_the_replay(oracle_lib, hostsim_lib):
    """A batch whose parallel pass is order-dependent is re-run (keyed chains or the one-lane replay): the
    trace holds the steps of the execution whose results the batch reports."""
    from test_async import batches, prog_mixed
    (u, d), = batches(1, 256, {0})
    pk = [3, 100, 128]
    maps = [(MapDef(MAP_ARRAY, 4, 16, 8), None)]
    a = _traced_run(hostsim_lib, prog_mixed(), maps, None, u, d, pk, 64)
    b = _traced_run(oracle_lib, prog_mixed(), maps, None, u, d, pk, 64)
    _same_trace(a[1], b[1], "replayed batch")
    assert a[0].stats["mode_used"] != MODE_PARALLEL


# ------------------------------------------------------------------------------------ helper table
def prog_host_helper(hid=100):
    """r1 = packet byte 0, r2 = 7, r3 = &stack, r4 = r5 = 0; call hid; r0 += 1; exit"""
    a = Asm()
    a.ldx(4, 6, 1, 0)
    a.ldx(1, 1, 6, 0)
    a.mov64(2, 7).mov64(3, src=10).add64(3, -8).mov64(4, 0).mov64(5, 0)
    a.call(hid)
    a.alu64(0x00, 0, 1).exit()
    return a.assemble()


class Recorder:
    """A host helper: R0 = 3 * R1 + packet; records (packet, args, kinds) in call order."""

    def __init__(self, fail_on=None):
        self.calls, self.fail_on = [], fail_on

    def __call__(self, packet, args, kinds):
        self.calls.append((packet, tuple(args), tuple(kinds)))
        if self.fail_on is not None and packet == self.fail_on:
            raise RuntimeError("helper error")
        return 3 * args[0] + packet


def _helper_run(lib, prog, umem, descs, hid=100, fail_on=None, settings=None):
    vm, _ = setup_one(lib, prog, [], settings)
    rec = Recorder(fail_on)
    vm.set_helper(hid, rec)
    r = vm.run_batch(umem.copy(), descs, want_regs=True)
    vm.close()
    return r, rec.calls


def test_host_helper_hostsim_equals_oracle(oracle_lib, hostsim_lib):
    umem, descs = packets(300, 64, seed=3)
    ra, ca = _helper_run(hostsim_lib, prog_host_helper(), umem, descs)
    rb, cb = _helper_run(oracle_lib, prog_host_helper(), umem, descs)
    assert ca == cb and [c[0] for c in cb] == list(range(300))  # every packet, in packet order
    assert (ra.results == rb.results).all() and (ra.regs == rb.regs).all()
    want = 3 * umem.reshape(300, 64)[:, 0].astype(np.int64) + np.arange(300) + 1
    assert (rb.results["r0"] == want).all()
    assert cb[0][2] == (IMM, IMM, FRAMEPTR, IMM, IMM) and cb[0][1][2] == -8  # a pointer passes its offset
    assert ra.stats["mode_used"] == MODE_SEQUENTIAL


def test_host_helper_error_aborts_the_packet(oracle_lib, hostsim_lib):
    umem, descs = packets(10, 64, seed=4)
    for lib in (oracle_lib, hostsim_lib):
        r, calls = _helper_run(lib, prog_host_helper(), umem, descs, fail_on=6)
        st = r.results
        assert st[6]["status"] == 1 and st[6]["code"] == E_HOST_HELPER | E_IN_HELPER  # VMERR
        assert (np.delete(st["status"], 6) == 0).all() and len(calls) == 10


def test_nil_and_replaced_builtin_helpers(oracle_lib, hostsim_lib):
    """HelperFunctions[1] = nil: the lookup fails with "no helper function" (inst_call_helper.go:26-28);
    HelperFunctions[14] replaced by a host function; reset_helper restores LinuxHelperFunctions."""
    a = Asm()
    a.call(14).mov64(6, src=0)
    a.mov64(1, 0).stx(4, 10, -4, 1).ld_map(1, 1).mov64(2, src=10).add64(2, -4).call(1)
    a.mov64(0, src=6).exit()
    prog = a.assemble()
    maps = [(MapDef(MAP_ARRAY, 4, 8, 4), None)]
    umem, descs = packets(5, 64)
    out = {}
    for name, lib in (("oracle", oracle_lib), ("hostsim", hostsim_lib)):
        vm, _ = setup_one(lib, prog, maps)
        vm.set_helper(1, None)
        r1 = vm.run_batch(umem.copy(), descs).results
        vm.reset_helper(1)
        vm.set_helper(14, lambda p, args, kinds: 1000 + p)
        r2 = vm.run_batch(umem.copy(), descs).results
        vm.reset_helper(14)
        r3 = vm.run_batch(umem.copy(), descs).results
        vm.close()
        assert (r1["status"] == 1).all() and (r1["code"] == 13).all()  # XE_E_NO_HELPER
        assert (r2["status"] == 0).all() and list(r2["r0"]) == [1000 + p for p in range(5)]
        assert (r3["r0"] == (1234 << 32) + 5678).all()
        out[name] = (r1, r2, r3)
    for x, y in zip(out["oracle"], out["hostsim"]):
        assert (x == y).all()


def test_helper_table_refuses_the_jit_engine(hostsim_lib):
    from gobpfld_amd.emulator import ENGINE_JIT
    vm, _ = setup_one(hostsim_lib, prog_host_helper(), [], Settings(engine=ENGINE_JIT))
    vm.set_helper(100, Recorder())
    umem, descs = packets(2, 64)
    with pytest.raises(EmulatorError):
        vm.run_batch(umem.copy(), descs)
    vm.close()


# ------------------------------------------------------------------------------------------ cancel
def _stream(lib, prog, bs, upto_sync, cancel_after):
    """Batches 0..upto_sync-1 synchronously, the rest pipelined, then xe_cancel."""
    vm = VM(Settings(), lib=lib)
    m = vm.add_map(MapDef(MAP_ARRAY, 4, 16, 8))
    vm.set_entrypoint(vm.add_raw_program(prog))
    keep, hs = [], []
    for b, (u, d) in enumerate(bs[:cancel_after]):
        u = u.copy()
        keep.append(u)
        if b < upto_sync:
            vm.run_batch_device(u.ctypes.data, u.nbytes, d.ctypes.data, len(d))
        else:
            hs.append(vm.run_batch_device_async(u.ctypes.data, u.nbytes, d.ctypes.data, len(d)))
    k = vm.cancel()
    dump = vm.map_dump(m)
    sts = [h._st.mode_used for h in hs]
    # the VM goes on from the surviving state
    u, d = bs[-1]
    u = u.copy()
    vm.run_batch_device(u.ctypes.data, u.nbytes, d.ctypes.data, len(d))
    after = vm.map_dump(m)
    vm.close()
    return k, dump, sts, after


def test_cancel_drops_pending_batches_hostsim(oracle_lib, hostsim_lib):
    from test_async import batches, oracle_stream, prog_mixed
    prog = prog_mixed()
    bs = batches(6, 256, set())
    k, dump, sts, after = _stream(hostsim_lib, prog, bs, upto_sync=2, cancel_after=5)
    _, want = oracle_stream(oracle_lib, prog, bs[:2])
    _, want_after = oracle_stream(oracle_lib, prog, bs[:2] + bs[-1:])
    assert k == 3 and dump == want and after == want_after
    assert sts == [MODE_CANCELLED] * 3
    vm = VM(Settings(), lib=hostsim_lib)
    assert vm.cancel() == 0  # nothing pending: a no-op
    vm.close()


# --------------------------------------------------------------------------------------------- GPU
@pytest.mark.gpu
@pytest.mark.parametrize("k", KATS[::3], ids=[k["name"] for k in KATS[::3]])
def test_trace_kats_device_equals_oracle(gpu_lib, oracle_lib, k):
    umem, descs = packets(256, k["pkt"], seed=7)
    pk = [0, 63, 64, 255]
    a = _traced_run(gpu_lib, k["program"], k["maps"], k["entries"], umem, descs, pk, 300)
    b = _traced_run(oracle_lib, k["program"], k["maps"], k["entries"], umem, descs, pk, 300)
    _same_trace(a[1], b[1], k["name"])
    assert (a[0].results == b[0].results).all()
    assert a[0].stats["engine_used"] == ENGINE_INTERP


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(8))
def test_trace_fuzz_device_equals_oracle(gpu_lib, oracle_lib, seed):
    prog, maps, entries, settings = gen_program(seed, 24 + seed % 64)
    umem, descs = packets(4096, 128, seed=seed)
    pk = list(range(0, 4096, 97))
    a = _traced_run(gpu_lib, prog, maps, entries, umem, descs, pk, 2000, settings)
    b = _traced_run(oracle_lib, prog, maps, entries, umem, descs, pk, 2000, settings)
    _same_trace(a[1], b[1], f"fuzz {seed}")


@pytest.mark.gpu
def test_host_helper_device_equals_oracle(gpu_lib, oracle_lib):
    """The device's one-lane replay calls the host function through the pinned mailbox, packet by packet."""
    umem, descs = packets(2000, 64, seed=3)
    ra, ca = _helper_run(gpu_lib, prog_host_helper(), umem, descs, fail_on=17)
    rb, cb = _helper_run(oracle_lib, prog_host_helper(), umem, descs, fail_on=17)
    assert ca == cb and len(cb) == 2000
    assert_same((ra, [], umem), (rb, [], umem), "host helper")
    assert ra.stats["mode_used"] == MODE_SEQUENTIAL


@pytest.mark.gpu
def test_cancel_device(gpu_lib):
    """Five pipelined 16M-packet C2 batches, then xe_cancel: the two the pipeline completed (its depth is
    three) stay, the other three are dropped; the map equals two batches' worth of counts."""
    import torch
    n = 16 * 1024 * 1024
    umem, descs = W.build_batch("c2", 0, n)
    d_umem = torch.from_numpy(umem).cuda()
    d_desc = torch.from_numpy(descs.view(np.uint8)).cuda()
    vm = VM(Settings(), lib=gpu_lib)
    W.setup_vm(vm, "c2")
    base = np.frombuffer(vm.map_dump(1), dtype=np.uint64).copy()
    vm.run_batch_device(d_umem.data_ptr(), d_umem.numel(), d_desc.data_ptr(), n)
    one = np.frombuffer(vm.map_dump(1), dtype=np.uint64) - base
    hs = [vm.run_batch_device_async(d_umem.data_ptr(), d_umem.numel(), d_desc.data_ptr(), n) for _ in range(5)]
    assert vm.cancel() == 3
    modes = [h._st.mode_used for h in hs]
    assert modes[:2] == [MODE_PARALLEL] * 2 and modes[2:] == [MODE_CANCELLED] * 3
    got = np.frombuffer(vm.map_dump(1), dtype=np.uint64)
    assert (got == base + 3 * one).all()
    vm.run_batch_device_async(d_umem.data_ptr(), d_umem.numel(), d_desc.data_ptr(), n).stats()
    assert (np.frombuffer(vm.map_dump(1), dtype=np.uint64) == base + 4 * one).all()
    vm.close()
