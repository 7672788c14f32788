"""The per-program kernel generator (JIT engine) on the CPU: the generated HIP source for every
BASELINE config and KAT compiles with hiprtc for gfx950 (no device needed to compile)."""
import ctypes as C

import numpy as np
import pytest

from gobpfld_amd import workloads as W
from kats import KATS


@pytest.fixture(scope="module")
def prod(built):
    from gobpfld_amd._native import PRODUCT_LIB
    lib = C.CDLL(str(PRODUCT_LIB))
    lib.xe_translate_uops.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32]
    lib.xe_jit_compile_check.argtypes = [C.c_void_p, C.c_size_t, C.c_char_p, C.c_size_t]
    lib.xe_jit_compile_check_keyed.argtypes = [C.c_void_p, C.c_size_t, C.c_char_p, C.c_size_t]
    lib.xe_jit_source.argtypes = [C.c_void_p, C.c_size_t, C.c_char_p, C.c_size_t]
    return lib


def _uops(lib, raw):
    raw = np.ascontiguousarray(np.asarray(raw, dtype=np.uint64))
    out = np.zeros(len(raw) * 16, dtype=np.uint8)
    n = lib.xe_translate_uops(raw.ctypes.data, len(raw), out.ctypes.data, len(raw))
    assert n >= 0
    return out, n


@pytest.mark.parametrize("name", ["c1", "c2", "c2rmw", "c3", "c4", "c5"])
def test_config_kernel_compiles(prod, name):
    u, n = _uops(prod, W.CONFIGS[name]["program"]())
    log = C.create_string_buffer(4096)
    assert prod.xe_jit_compile_check(u.ctypes.data, n, log, 4096) == 0, log.value.decode()


@pytest.mark.parametrize("name", ["c2rmw", "c3learn", "c5"])
def test_keyed_variant_compiles(prod, name):
    """The keyed variant (XE_MODE_SPEC / XE_MODE_CHAIN, xe_internal.h) of the per-program kernel."""
    u, n = _uops(prod, W.CONFIGS[name]["program"]())
    log = C.create_string_buffer(4096)
    assert prod.xe_jit_compile_check_keyed(u.ctypes.data, n, log, 4096) == 0, log.value.decode()


def test_kat_kernels_compile(prod):
    # one combined pass keeps the CPU suite fast: compile a handful of structurally different KATs
    names = {"jump_negative_panics", "budget_exhausted", "hash_key_readrange_rounding", "callx_dispatch",
             "fallthrough_bad_pc", "ld_abs_not_implemented", "unaligned_xadd_on_array", "lddw_map_value"}
    for k in KATS:
        if k["name"] not in names:
            continue
        u, n = _uops(prod, k["program"])
        log = C.create_string_buffer(4096)
        assert prod.xe_jit_compile_check(u.ctypes.data, n, log, 4096) == 0, (k["name"], log.value.decode())


def test_generated_source_shape(prod):
    u, n = _uops(prod, W.CONFIGS["c2"]["program"]())
    buf = C.create_string_buffer(1 << 20)
    prod.xe_jit_source(u.ctypes.data, n, buf, 1 << 20)
    src = buf.value.decode()
    assert "#define XE_REGS_FIELDS" in src and "xe_jit_kernel" in src
    assert src.count("\nL") >= n            # one labelled block per instruction slot
    assert "steps >= P.max_steps" not in src.split("XE_DEV void xe_jit_body")[1].split("L0:")[1].split("L1:")[0]


def test_kernel_cache_fill(prod, tmp_path):
    """gobpfld_amd/kcache.py: worker processes compile generated sources into the on-disk kernel cache
    (xe_compile_kernel_source, no device); one object per distinct source, named by the content hash
    (a changed source gets a new object), and a second fill finds everything cached."""
    from gobpfld_amd import kcache
    srcs = []
    for name in ("c1", "c2", "c4"):
        u, n = _uops(prod, W.CONFIGS[name]["program"]())
        buf = C.create_string_buffer(1 << 21)
        prod.xe_jit_source(u.ctypes.data, n, buf, 1 << 21)
        srcs.append(buf.value.decode())
    srcs.append(srcs[0])                                      # duplicates compile once
    assert kcache.fill(srcs, tmp_path, workers=3) == []
    objs = sorted(p.name for p in tmp_path.glob("xe_*.co"))
    assert len(objs) == 3 and all(len(p) == len("xe_") + 32 + len(".co") for p in objs)
    mtimes = {p.name: p.stat().st_mtime_ns for p in tmp_path.glob("xe_*.co")}
    assert kcache.fill(srcs[:1] + [srcs[1] + "\n// changed\n"], tmp_path, workers=2) == []
    after = {p.name: p.stat().st_mtime_ns for p in tmp_path.glob("xe_*.co")}
    assert len(after) == 4 and all(after[k] == v for k, v in mtimes.items())
    assert kcache.fill(["this is not HIP"], tmp_path, workers=1)   # a compile error is reported
