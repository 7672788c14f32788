"""Key shadows (xe_jit.cpp key_shadows): a per-program kernel hands a HASH lookup / update the key
words it built from the values it stored into the frame instead of walking ReadRange(R2, key_size)
(xe_interp.h read_key), where the generator proves the two equal.

CPU: which key constructions the generator accepts (the generated source of a host-simulation VM).
GPU: every construction — accepted or refused, including the ReadRange quirks the proof has to respect
(a store straddling the key's first byte, a partly overwritten store, an object changed through an
aliasing register) — gives the oracle's results, registers and final map on the device."""
from __future__ import annotations

import numpy as np
import pytest

from gobpfld_amd.asm import JEQ, JGT, Asm
from gobpfld_amd.emulator import MAP_ARRAY, MAP_HASH, MapDef, Settings

JIT = 2
NKEYS = 16


def _head(a: Asm) -> None:
    a.ldx(4, 6, 1, 0).ldx(4, 7, 1, 4)          # data, data_end
    a.mov64(2, src=6).add64(2, 32)
    a.jmp(JGT, 2, "out", src=7)


def _tail(a: Asm, helper: int = 1) -> None:
    a.ld_map(1, 1)
    a.mov64(2, src=10).add64(2, -16)
    if helper == 2:
        a.ldx(8, 3, 6, 16).stx(8, 10, -32, 3)   # value = packet bytes 16..23
        a.mov64(3, src=10).add64(3, -32)
        a.mov64(4, 0)
        a.call(2)
        a.exit()                                # R0 = the update's errno
    else:
        a.call(1)
    a.label("after")
    a.jmp(JEQ, 0, "miss", imm=0)
    a.mov64(1, 1).xadd(8, 0, 0, 1)              # count the hit in the value
    a.ldx(8, 0, 0, 0)
    a.exit()
    a.label("miss")
    a.mov64(0, 2)
    a.exit()
    a.label("out")
    a.mov64(0, 1)
    a.exit()


def k_tuple(a):  # C5's 5-tuple key: seven stores of 4 / 4 / 2 / 2 / 1 / 1 / 2 bytes
    a.ldx(4, 3, 6, 0).stx(4, 10, -16, 3)
    a.ldx(4, 3, 6, 4).stx(4, 10, -12, 3)
    a.ldx(2, 3, 6, 8).stx(2, 10, -8, 3)
    a.ldx(2, 3, 6, 10).stx(2, 10, -6, 3)
    a.ldx(1, 3, 6, 12).stx(1, 10, -4, 3)
    a.st(1, 10, -3, 0).st(2, 10, -2, 0)


def k_wide(a):
    a.ldx(8, 3, 6, 0).stx(8, 10, -16, 3)
    a.ldx(8, 4, 6, 8).stx(8, 10, -8, 4)


def k_via_ptr(a):  # stores through a copy of R10 moved by immediates
    a.mov64(5, src=10).add64(5, -40).add64(5, 24)
    a.ldx(8, 3, 6, 0).stx(8, 5, 0, 3)
    a.ldx(4, 3, 6, 8).stx(4, 5, 8, 3)
    a.ldx(4, 3, 6, 12).stx(4, 5, 12, 3)


def k_negimm(a):  # ST immediates are sign-extended objects; the key takes their low bytes
    a.st(4, 10, -16, -2).st(2, 10, -12, -3).st(2, 10, -10, 0x7ff)
    a.ldx(8, 3, 6, 0).stx(8, 10, -8, 3)


def k_split(a):  # the key is stored in one block, looked up in the next (its only predecessor)
    k_wide(a)
    a.ldx(1, 3, 6, 20)
    a.jmp(JEQ, 3, "out", imm=0x5a)


def k_straddle(a):  # an 8-byte store over the key's first byte: ReadRange reads its low 4 bytes
    a.ldx(8, 3, 6, 0).stx(8, 10, -20, 3)
    a.ldx(4, 3, 6, 8).stx(4, 10, -12, 3)
    a.ldx(8, 3, 6, 8).stx(8, 10, -8, 3)


def k_overwrite(a):  # a byte of an 8-byte store overwritten: the rest reads as 4-byte runs of it
    k_wide(a)
    a.st(1, 10, -13, 0x55)


def k_alias(a):  # LDX makes R4 alias the stored object; the in-place add changes the key (all 8 bytes)
    k_wide(a)
    a.ldx(4, 4, 10, -16)
    a.add64(4, 1)


def k_alias_ldimm(a):  # LD_IMM64 (src 0) assigns in place (inst_load.go:65): the aliased object takes it
    k_wide(a)
    a.ldx(8, 4, 10, -16)
    a.ld_imm64(4, 0x1122334455667788)


def k_alias_replaced(a):  # ADD of a pointer replaces R4 instead (inst_add.go:82-98): the object stays
    k_wide(a)
    a.ldx(4, 4, 10, -16)
    a.add64(4, src=6)


def k_unwritten(a):  # the last four key bytes were never written (object 0 reads as zero)
    a.ldx(8, 3, 6, 0).stx(8, 10, -16, 3)
    a.ldx(4, 3, 6, 8).stx(4, 10, -8, 3)


def k_two_preds(a):  # the lookup block has two predecessors: no proof
    a.ldx(1, 3, 6, 20)
    a.jmp(JEQ, 3, "b", imm=0x5a)
    k_wide(a)
    a.ja("look")
    a.label("b")
    k_wide(a)
    a.label("look")


def k_readback(a):  # a frame load besides the key: the key is still shadowed, the stores stay
    k_wide(a)
    a.ldx(8, 5, 10, -16)


def k_helper_between(a):  # another helper call between the stores and the lookup
    k_wide(a)
    a.call(14)


# name -> (key builder, helper, key size, generator accepts it, key of a packet for the preloaded entries)
CASES = {
    "tuple": (k_tuple, 1, 16, True, lambda p: p[0:13] + b"\0\0\0"),
    "wide": (k_wide, 1, 16, True, lambda p: p[0:16]),
    "via_ptr": (k_via_ptr, 1, 16, True, lambda p: p[0:16]),
    "negimm": (k_negimm, 1, 16, True, lambda p: b"\xfe\xff\xff\xff\xfd\xff\xff\x07" + p[0:8]),
    "split": (k_split, 1, 16, True, lambda p: p[0:16]),
    "readback": (k_readback, 1, 16, True, lambda p: p[0:16]),
    "update": (k_wide, 2, 16, True, None),
    "straddle": (k_straddle, 1, 16, False, lambda p: p[0:4] + p[8:12] + p[8:16]),
    "overwrite": (k_overwrite, 1, 16, False, lambda p: p[0:4] + p[0:4] + p[8:16]),
    "alias": (k_alias, 1, 16, True, lambda p: ((int.from_bytes(p[0:8], "little") + 1) % 2**64).to_bytes(8, "little") + p[8:16]),
    "alias_ldimm": (k_alias_ldimm, 1, 16, True, lambda p: (0x1122334455667788).to_bytes(8, "little") + p[8:16]),
    "alias_replaced": (k_alias_replaced, 1, 16, False, lambda p: p[0:16]),
    "unwritten": (k_unwritten, 1, 16, False, lambda p: p[0:12] + b"\0\0\0\0"),
    "two_preds": (k_two_preds, 1, 16, False, lambda p: p[0:16]),
    "helper_between": (k_helper_between, 1, 16, False, lambda p: p[0:16]),
    "array_map": (k_wide, 1, 4, False, None),
}


# the cases whose frame stores the kernel leaves out (xe_jit.cpp dead_frame_stores): the frame is only
# read through shadowed keys
NO_STORES = {"tuple", "wide", "via_ptr", "negimm", "split"}


def program(name: str) -> list[int]:
    build, helper, _, _, _ = CASES[name]
    a = Asm()
    _head(a)
    build(a)
    _tail(a, helper)
    return a.assemble()


def packets(n: int, seed: int = 5):
    """n 64-byte packets whose first 16 bytes come from a pool of NKEYS patterns (lookups hit)"""
    from gobpfld_amd._native import np_dtypes
    d_desc, _, _ = np_dtypes()
    rng = np.random.default_rng(seed)
    pool = rng.integers(0, 256, size=(NKEYS, 16), dtype=np.uint8)
    pk = rng.integers(0, 256, size=(n, 64), dtype=np.uint8)
    pk[:, :16] = pool[rng.integers(0, NKEYS, size=n)]
    descs = np.zeros(n, dtype=d_desc)
    descs["addr"] = np.arange(n) * 64
    descs["len"] = 64
    return pk.reshape(-1).copy(), descs, pool


def case(name: str, pool=None):
    """(program, maps, entries) of a case; entries: half the pool's keys, as the case builds them"""
    _, _, ks, _, keyfn = CASES[name]
    if name == "array_map":
        return program(name), [(MapDef(MAP_ARRAY, 4, 8, 64), None)], None
    ents = None
    if keyfn is not None and pool is not None:
        ents = {0: [(keyfn(bytes(pool[i]) + bytes(8)), (1000 * (i + 1)).to_bytes(8, "little")) for i in range(0, NKEYS, 2)]}
    return program(name), [(MapDef(MAP_HASH, ks, 8, 256), None)], ents


def kernel_cases():
    """(program, maps, entries, settings) of every case, for the suite's kernel precompile"""
    _, _, pool = packets(8)
    return [(*case(name, pool), Settings(engine=JIT)) for name in CASES]


def _source(hostsim_lib, name: str) -> str:
    from gobpfld_amd import aot
    _, _, pool = packets(8)
    srcs = aot.sources([(*case(name, pool), Settings(engine=JIT))], lib=hostsim_lib, variants=(0,))
    assert len(srcs) == 1
    return srcs[0]


@pytest.mark.parametrize("name", sorted(CASES))
def test_generator_accepts_exactly_the_proven_keys(hostsim_lib, name):
    src = _source(hostsim_lib, name).split("XE_DEV void xe_jit_body")[1]
    assert src.count("uop_helper_key(L") == (1 if CASES[name][3] else 0), name
    assert (src.count("uop_store(") == 0) == (name in NO_STORES), name


def test_config_kernels_use_key_shadows(hostsim_lib):
    """C3 and C5 look their 5-tuple up through a key shadow and store nothing into the frame; C3-learn's
    update too, with its key's saddr object changed in place through an aliasing register before the call
    (emulator/memory.go:37-52): the shadow takes the register's new value."""
    from gobpfld_amd import aot
    from gobpfld_amd import workloads as W
    for name, sites in (("c3", 1), ("c5", 1), ("c3learn", 2), ("c2", 0), ("bpf2bpf", 0)):
        srcs = aot.sources([lambda vm, n=name: W.setup_vm(vm, n)], lib=hostsim_lib, variants=(0,))
        body = srcs[0].split("XE_DEV void xe_jit_body")[1]
        assert body.count("uop_helper_key(L") == sites, name
        if name in ("c3", "c5"):
            assert body.count("uop_store(") == 0, name


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(CASES))
def test_key_shadow_device_equals_oracle(gpu_lib, oracle_lib, name):
    from parity import assert_same, run_one
    umem, descs, pool = packets(4096)
    prog, maps, entries = case(name, pool)
    a = run_one(gpu_lib, prog, maps, umem, descs, entries=entries, settings=Settings(engine=JIT))
    b = run_one(oracle_lib, prog, maps, umem, descs, entries=entries)
    assert a[0].stats["engine_used"] == JIT, "the per-program kernel must run"
    assert_same(a, b, name)
    if CASES[name][4] is not None:  # the preloaded keys are found: the key bytes matter
        assert (b[0].results["r0"] > 1000).any(), name
