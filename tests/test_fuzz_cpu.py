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
