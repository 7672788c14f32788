"""Differential fuzzing on CPU: random programs (tests/fuzz.py) through the product's translator and
interpreter compiled for the host (XE_HOSTSIM build of the same xe_interp.h the GPU runs) against the
oracle. Bit-exact on every observable (tests/parity.py:assert_same)."""
import numpy as np
import pytest

from fuzz import gen_program
from parity import assert_same, run_one


def fuzz_packets(seed: int, n: int = 48):
    from gobpfld_amd._native import np_dtypes
    d_desc, _, _ = np_dtypes()
    rng = np.random.default_rng(seed ^ 0x5EED)
    lens = rng.choice([0, 1, 13, 14, 20, 34, 54, 60, 64, 100], size=n)
    offs = np.concatenate([[0], np.cumsum(lens + 8)[:-1]]).astype(np.int64)
    umem = rng.integers(0, 256, size=int(offs[-1] + lens[-1] + 8), dtype=np.uint8)
    descs = np.zeros(n, dtype=d_desc)
    descs["addr"] = offs
    descs["len"] = lens
    return umem, descs


def _try(lib, prog, maps, entries, umem, descs, settings):
    try:
        return run_one(lib, prog, maps, umem, descs, settings=settings, entries=entries), None
    except Exception as e:  # decode/translate rejection must match too
        return None, str(e).split(":")[0]


@pytest.mark.parametrize("block", range(8))
def test_fuzz_hostsim_equals_oracle(oracle_lib, hostsim_lib, block):
    statuses = np.zeros(8, dtype=np.int64)
    for seed in range(block * 60, block * 60 + 60):
        prog, maps, entries, settings = gen_program(seed)
        umem, descs = fuzz_packets(seed)
        a, ea = _try(hostsim_lib, prog, maps, entries, umem, descs, settings)
        b, eb = _try(oracle_lib, prog, maps, entries, umem, descs, settings)
        assert (a is None) == (b is None), (seed, ea, eb)
        if a is None:
            continue
        assert_same(a, b, f"fuzz seed {seed}")
        statuses += np.bincount(b[0].results["status"], minlength=8)[:8]
    # the generator must reach normal exits and error paths alike
    assert statuses[0] > 0 and statuses[1] > 0, statuses


def _may_write(lib, prog):
    import ctypes as C
    arr = np.ascontiguousarray(np.asarray(prog, dtype=np.uint64))
    fn = lib.dll.xe_debug_may_write_packet
    fn.restype = C.c_int
    fn.argtypes = [C.c_void_p, C.c_uint32]
    return fn(arr.ctypes.data, len(arr))


def test_packet_write_analysis_is_sound(oracle_lib, hostsim_lib):
    """Programs the analysis clears never change packet bytes in the oracle; the configs are cleared."""
    from gobpfld_amd import workloads as W
    for name in ("c1", "c2", "c3", "c4", "c5"):
        assert _may_write(hostsim_lib, W.CONFIGS[name]["program"]()) == 0, name
    cleared = flagged = 0
    for seed in range(600):
        prog, maps, entries, settings = gen_program(seed)
        umem, descs = fuzz_packets(seed)
        verdict = _may_write(hostsim_lib, prog)
        assert verdict in (0, 1)
        b, _ = _try(oracle_lib, prog, maps, entries, umem, descs, settings)
        if verdict == 0:
            cleared += 1
            assert np.array_equal(b[2], umem), f"seed {seed}: packet written but analysis cleared it"
        else:
            flagged += 1
    assert cleared > 50 and flagged > 50, (cleared, flagged)
