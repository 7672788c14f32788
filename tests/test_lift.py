"""Read-modify-write lifting (xe_runtime.cpp lift_rmw; uop_ldx / uop_store in xe_interp.h).

`ldx rX, [rB+o]; add/sub rX, K|rY; stx [rB+o], rX` with rX dead afterwards is what `value->count++`
compiles to without an atomic. Sequentially it is an add; a parallel lane runs it as one, so such
programs stay in the parallel mode instead of conflicting into the ordered replay. The results must
still equal the oracle's sequential VM bit for bit, and the pattern must not be lifted where the loaded
value stays observable (a later use, a register record, a jump into the middle, a non-add update)."""
import ctypes as C

import numpy as np
import pytest

from gobpfld_amd import workloads as W
from gobpfld_amd.asm import ADD, JEQ, MUL, Asm
from gobpfld_amd.emulator import MAP_ARRAY, MODE_KEYED, MODE_PARALLEL, MODE_SEQUENTIAL, MapDef, Settings
from parity import assert_same, config_case, packets, run_one

UF_LIFT = 0x40


def _lifted(raw):
    """Instruction indices whose micro-op carries UF_LIFT (LDX and STX of lifted pairs)."""
    from gobpfld_amd.build import HOSTSIM_LIB
    lib = C.CDLL(str(HOSTSIM_LIB))
    lib.xe_translate_uops.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32]
    raw = np.ascontiguousarray(np.asarray(raw, dtype=np.uint64))
    out = np.zeros((len(raw), 16), dtype=np.uint8)
    n = lib.xe_translate_uops(raw.ctypes.data, len(raw), out.ctypes.data, len(raw))
    assert n == len(raw)
    return [i for i in range(n) if out[i, 3] & UF_LIFT]


def _prog(variant):
    """Key = packet byte 0 & 7 into an ARRAY(8 x 16 B); then one update of the looked-up value."""
    a = Asm()
    a.ldx(4, 6, 1, 0)                      # r6 = data
    a.ldx(1, 8, 6, 0).alu64(0x50, 8, 7)    # r8 = byte 0 & 7
    a.ldx(1, 9, 6, 1)                      # r9 = byte 1
    a.stx(4, 10, -4, 8).ld_map(1, 1).mov64(2, src=10).add64(2, -4).call(1)
    a.jmp(JEQ, 0, "out", imm=0)
    if variant == "add_imm64":
        a.ldx(8, 1, 0, 0).add64(1, 3).stx(8, 0, 0, 1)
    elif variant == "sub_reg64":
        a.ldx(8, 2, 0, 8).sub64(2, src=9).stx(8, 0, 8, 2)
    elif variant == "add32_reg_w4":
        a.ldx(4, 3, 0, 4).alu32(ADD, 3, src=8).stx(4, 0, 4, 3)
    elif variant == "two_fields":
        a.ldx(8, 1, 0, 0).add64(1, 1).stx(8, 0, 0, 1)
        a.ldx(8, 1, 0, 8).add64(1, src=9).stx(8, 0, 8, 1)
    elif variant == "used_after":          # the loaded sum becomes the verdict: stays ordered
        a.ldx(8, 1, 0, 0).add64(1, 1).stx(8, 0, 0, 1).mov64(0, src=1).alu64(0x50, 0, 3).exit()
    elif variant == "other_read":          # lifted add, then a plain read of the same field: conflict
        a.ldx(8, 1, 0, 0).add64(1, 1).stx(8, 0, 0, 1).ldx(8, 0, 0, 0).alu64(0x50, 0, 3).exit()
    elif variant == "mul":                 # not an add: stays ordered
        a.ldx(8, 1, 0, 0).alu64(MUL, 1, 3).stx(8, 0, 0, 1)
    a.label("out").mov64(0, 2).exit()
    return a.assemble()


LIFTED = ["add_imm64", "sub_reg64", "add32_reg_w4", "two_fields"]
ORDERED = ["used_after", "other_read", "mul"]


def _mode(variant, parallel, regs=False):
    """Lifted: parallel. A plain store into the value (not lifted): keyed ordered execution (chains per
    written key). other_read, lifted (no register records): a plain read of a field other lanes add to,
    the one-lane replay."""
    if parallel:
        return MODE_PARALLEL
    return MODE_SEQUENTIAL if variant == "other_read" and not regs else MODE_KEYED


def test_lift_static_pattern():
    c2 = _lifted(W.CONFIGS["c2rmw"]["program"]())
    assert len(c2) == 2 and c2[1] == c2[0] + 2
    assert _lifted(W.CONFIGS["c2"]["program"]()) == []
    for v in LIFTED:
        assert len(_lifted(_prog(v))) == (4 if v == "two_fields" else 2), v
    assert _lifted(_prog("used_after")) == [] and _lifted(_prog("mul")) == []
    assert len(_lifted(_prog("other_read"))) == 2  # lifted; the later plain read conflicts at run time

    def variant(edit):
        a = Asm()
        a.ld_map_value(6, 1)
        edit(a)
        a.mov64(0, 2).exit()
        return _lifted(a.assemble())
    assert variant(lambda a: a.ldx(8, 1, 6, 0).add64(1, 1).stx(8, 6, 0, 1)) == [2, 4]
    assert variant(lambda a: a.ldx(8, 1, 6, 0).add64(1, 1).stx(8, 6, 8, 1)) == []       # other offset
    assert variant(lambda a: a.ldx(8, 1, 6, 0).alu32(ADD, 1, 1).stx(8, 6, 0, 1)) == []  # 32-bit add, 8-B store
    assert variant(lambda a: a.ldx(4, 1, 6, 0).add64(1, src=1).stx(4, 6, 0, 1)) == []   # addend is the load
    assert variant(lambda a: a.ldx(2, 1, 6, 0).add64(1, 1).stx(2, 6, 0, 1)) == []       # no 2-B lifting
    assert variant(lambda a: a.ldx(8, 6, 6, 0).add64(6, 1).stx(8, 6, 0, 6)) == []       # base = loaded reg

    def jump_into_middle():
        a = Asm()
        a.ld_map_value(6, 1).mov64(1, 0)
        a.jmp(JEQ, 1, "mid", imm=1)
        a.ldx(8, 1, 6, 0).label("mid").add64(1, 1).stx(8, 6, 0, 1)
        a.mov64(0, 2).exit()
        return _lifted(a.assemble())
    assert jump_into_middle() == []

    def with_call(callee_reads_r1: bool, caller_reads_r1: bool = False):
        a = Asm()
        a.ld_map_value(6, 1).ldx(8, 1, 6, 0).add64(1, 1).stx(8, 6, 0, 1)
        a.call_bpf("f")
        if caller_reads_r1:
            a.mov64(0, src=1).exit()
        else:
            a.mov64(0, 2).exit()
        a.label("f")
        a.mov64(0, src=1) if callee_reads_r1 else a.mov64(0, 0)
        a.exit()
        return _lifted(a.assemble())
    # liveness follows the call into the callee and, past its exit, to the return site
    assert with_call(False) == [2, 4]
    assert with_call(True) == []           # R1 is the callee's argument
    assert with_call(False, True) == []    # R1 survives the return (R0..R5 are not restored)


def _maps():
    return [(MapDef(MAP_ARRAY, 4, 16, 8), None)]


@pytest.mark.parametrize("variant", LIFTED + ORDERED)
@pytest.mark.parametrize("regs", [False, True], ids=["noregs", "regs"])
def test_lift_hostsim_equals_oracle(oracle_lib, hostsim_lib, variant, regs):
    umem, descs = packets(2048, 64, seed=11)
    a = run_one(hostsim_lib, _prog(variant), _maps(), umem, descs, regs=regs)
    b = run_one(oracle_lib, _prog(variant), _maps(), umem, descs, regs=regs)
    assert_same(a, b, variant)
    parallel = variant in LIFTED and not regs
    assert a[0].stats["mode_used"] == _mode(variant, parallel, regs), variant
    assert a[0].stats["conflict"] == (0 if parallel else 1), variant


def test_c2rmw_hostsim_parallel(oracle_lib, hostsim_lib):
    prog, maps, entries, umem, descs = config_case("c2rmw", 16384)
    a = run_one(hostsim_lib, prog, maps, umem, descs, entries=entries, regs=False)
    b = run_one(oracle_lib, prog, maps, umem, descs, entries=entries, regs=False)
    assert_same(a, b, "c2rmw")
    assert a[0].stats["mode_used"] == MODE_PARALLEL and a[0].stats["conflict"] == 0
    c2 = run_one(oracle_lib, *config_case("c2", 16384)[:2], umem, descs, regs=False)
    assert a[1] == c2[1], "the lifted counters must equal C2's atomic ones"


@pytest.mark.gpu
@pytest.mark.parametrize("engine", [1, 2], ids=["interp", "jit"])
@pytest.mark.parametrize("variant", LIFTED + ORDERED)
def test_lift_device_equals_oracle(gpu_lib, oracle_lib, variant, engine):
    umem, descs = packets(30000, 64, seed=12)
    a = run_one(gpu_lib, _prog(variant), _maps(), umem, descs, regs=False, settings=Settings(engine=engine))
    b = run_one(oracle_lib, _prog(variant), _maps(), umem, descs, regs=False)
    assert_same(a, b, variant)
    assert a[0].stats["mode_used"] == _mode(variant, variant in LIFTED), variant


@pytest.mark.gpu
@pytest.mark.parametrize("engine", [1, 2], ids=["interp", "jit"])
def test_c2rmw_device_parallel(gpu_lib, oracle_lib, engine):
    prog, maps, entries, umem, descs = config_case("c2rmw", 1 << 20)
    a = run_one(gpu_lib, prog, maps, umem, descs, entries=entries, regs=False, settings=Settings(engine=engine))
    b = run_one(oracle_lib, prog, maps, umem, descs, entries=entries, regs=False)
    assert_same(a, b, "c2rmw")
    assert a[0].stats["mode_used"] == MODE_PARALLEL and a[0].stats["conflict"] == 0


def test_lift_through_bpf_to_bpf_calls(oracle_lib, hostsim_lib):
    """lift_rmw follows bpf-to-bpf calls (a call flows into its callee and on to the return site): the
    `stats->pkts++` / `stats->bytes += size` inside workloads.prog_bpf2bpf's callee are lifted, so the
    batch runs in parallel and still equals the oracle's sequential VM."""
    prog, maps, entries, umem, descs = config_case("bpf2bpf", 2000)
    a = run_one(hostsim_lib, prog, maps, umem, descs, entries=entries, regs=False)
    b = run_one(oracle_lib, prog, maps, umem, descs, entries=entries, regs=False)
    assert_same(a, b, "bpf2bpf")
    assert a[0].stats["mode_used"] == 1, a[0].stats
    from gobpfld_amd import _native as N
    import ctypes as C
    lib = C.CDLL(str(N.PRODUCT_LIB))
    raw = np.ascontiguousarray(np.asarray(prog, dtype=np.uint64))
    out = np.zeros(len(raw) * 16, dtype=np.uint8)
    n = lib.xe_translate_uops(raw.ctypes.data_as(C.c_void_p), len(raw), out.ctypes.data_as(C.c_void_p), len(raw))
    fl = out.reshape(-1, 16)[:n, 3]
    assert int(((fl & 0x40) != 0).sum()) == 4     # two load/store pairs in the callee
