"""Step totals of the verdict-only kernel variant (xe_jit.cpp XE_JV_LEAN, the block form of
emit_body_blocks): a verdict-only batch reports no per-packet records, only the batch's step total (the
instructions every packet retired, emulator/vm.go:117-173 counts each one up to and including the exit or
the failing instruction) and its status histogram. These runs compare both, and the verdicts, with the
oracle's sequential VM: C4's ACL chain at the benchmark's geometry, and a program whose regions fail
part-way (an unchecked packet read past the end of short packets) and whose jump chain closes a region.
(Round 6 measured counting these steps per wave on the scalar unit: C4 0.632 ms against 0.609 — the
scalar unit issues at the same rate per SIMD as the vector one, and the counts cost more scalar
instructions than the selects they replaced. Not kept.)"""
import numpy as np
import pytest

from gobpfld_amd import workloads as W
from gobpfld_amd.asm import JEQ, JGT, Asm
from gobpfld_amd.emulator import ENGINE_JIT, VM, Settings


def prog_rules_with_errors():
    """r3 = packet[0]: 36 JEQ rules (the block form's if-converted chain); then a region that reads
    packet[40] without a bounds check (an error on packets of 40 bytes or less), adds it to R0 and ends
    in a jump chain on it (JEQ, JEQ, JGT, JA)."""
    a = Asm()
    a.ldx(4, 6, 1, 0)
    a.mov64(0, 1)
    a.ldx(1, 3, 6, 0)
    for i in range(36):
        a.jmp(JEQ, 3, "hit", imm=7 * i + 1)
    a.ldx(1, 4, 6, 40)
    a.add64(0, src=4)
    a.jmp(JEQ, 4, "hit", imm=5)
    a.jmp(JEQ, 4, "hit", imm=9)
    a.jmp(JGT, 4, "hit", imm=200)
    a.ja("out")
    a.label("hit").mov64(0, 2).exit()
    a.label("out").mov64(0, 3).exit()
    return a.assemble()


def error_batch(n: int, seed: int = 5):
    """n packets of 16..64 bytes (random contents), back to back"""
    from gobpfld_amd._native import np_dtypes
    d_desc, _, _ = np_dtypes()
    rng = np.random.default_rng(seed)
    lens = rng.integers(16, 65, size=n)
    addr = np.zeros(n, dtype=np.uint64)
    addr[1:] = np.cumsum(lens)[:-1]
    umem = rng.integers(0, 256, size=int(lens.sum()), dtype=np.uint8)
    descs = np.zeros(n, dtype=d_desc)
    descs["addr"] = addr
    descs["len"] = lens
    return umem, descs


def setup_errors(vm):
    vm.set_entrypoint(vm.add_raw_program(prog_rules_with_errors()))


def _setup(vm, case):
    if case == "c4":
        W.setup_vm(vm, "c4")
    else:
        setup_errors(vm)


def _batch(case, n):
    return W.build_batch("c4", 0, n) if case == "c4" else error_batch(n)


def test_error_program_hostsim_equals_oracle(hostsim_lib, oracle_lib):
    """The program's statuses and steps in the host simulation (the reference for the device test)."""
    from parity import assert_same, run_one
    umem, descs = error_batch(4096)
    got = run_one(hostsim_lib, prog_rules_with_errors(), [], umem, descs)
    want = run_one(oracle_lib, prog_rules_with_errors(), [], umem, descs)
    assert_same(got, want, "errors")
    status = want[0].results["status"]
    assert 0.1 < (status != 0).mean() < 0.7  # both outcomes well represented


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["c4", "errors"])
def test_verdict_only_steps_equal_oracle(oracle_lib, case):
    import torch
    n = 65536
    umem, descs = _batch(case, n)
    ov = VM(Settings(), lib=oracle_lib)
    _setup(ov, case)
    ro = ov.run_batch(umem.copy(), descs)
    ov.close()
    d_umem = torch.from_numpy(umem.copy()).cuda()
    d_desc = torch.from_numpy(descs.view(np.uint8)).cuda()
    d_ver = torch.zeros(n, dtype=torch.int32, device="cuda")
    vm = VM(Settings())
    _setup(vm, case)
    vm.prepare()
    st = vm.run_batch_device(d_umem.data_ptr(), d_umem.numel(), d_desc.data_ptr(), n, d_verdicts=d_ver.data_ptr())
    torch.cuda.synchronize()
    vm.close()
    assert st["engine_used"] == ENGINE_JIT, st  # the per-program kernel (its verdict-only variant)
    assert (d_ver.cpu().numpy().view(np.uint32) == ro.verdicts).all(), "verdicts differ"
    want_hist = np.bincount(ro.results["status"], minlength=8)[:8]
    assert list(st["status_count"][:8]) == list(want_hist), (st["status_count"], want_hist)
    assert st["steps"] == ro.stats["steps"], (st["steps"], ro.stats["steps"])
