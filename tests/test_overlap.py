"""Descriptors whose bytes overlap, with a program that writes packets.

The reference walks the packets in order (emulator/vm.go:110-173 per packet), so a
packet whose bytes an earlier packet of the batch also covers reads what that packet wrote. Parallel
lanes cannot reproduce that: the runtime checks the descriptors of a packet-writing program (sorted
byte ranges, exact) and runs such a batch in order. Every case must equal the oracle's single VM —
verdicts, R0..R9 records and the packet bytes left in the UMEM."""
import numpy as np
import pytest

from gobpfld_amd._native import np_dtypes
from gobpfld_amd.asm import Asm
from gobpfld_amd.emulator import MODE_PARALLEL, MODE_SEQUENTIAL, Settings
from parity import assert_same, run_one


def prog_bump():
    """pkt[4] += 1 (a byte store into the packet); return the new value."""
    a = Asm()
    a.ldx(4, 2, 1, 0)            # r2 = data
    a.ldx(1, 3, 2, 4).add64(3, 1)
    a.stx(1, 2, 4, 3)
    a.mov64(0, src=3).exit()
    return a.assemble()


def layout(kind: str, n: int = 256):
    d_desc, _, _ = np_dtypes()
    umem = np.zeros(64 * n, dtype=np.uint8)
    descs = np.zeros(n, dtype=d_desc)
    descs["len"] = 64
    if kind == "disjoint":          # back to back: no byte shared
        descs["addr"] = np.arange(n) * 64
    elif kind == "same":            # every descriptor on the same 64 bytes
        descs["addr"] = 0
    elif kind == "shifted":         # packet i at 32 * i: each shares half of its bytes with the next
        descs["addr"] = np.arange(n) * 32
    elif kind == "pairs":           # two descriptors per frame, in a shuffled order
        rng = np.random.default_rng(7)
        descs["addr"] = rng.permutation(np.repeat(np.arange(n // 2) * 64, 2))
    elif kind == "touching":        # [a, a + 60) then [a + 60, ...): adjacent, never shared
        descs["addr"] = np.arange(n) * 60
        descs["len"] = 60
    return umem, descs


KINDS = [("disjoint", False), ("same", True), ("shifted", True), ("pairs", True), ("touching", False)]


def _check(lib, oracle_lib, kind, overlapping):
    umem, descs = layout(kind)
    prog = prog_bump()
    got = run_one(lib, prog, [], umem, descs)
    want = run_one(oracle_lib, prog, [], umem, descs)
    assert_same(got, want, kind)
    assert (got[2] == want[2]).all(), f"{kind}: packet bytes differ"
    mode = got[0].stats["mode_used"]
    assert mode == (MODE_SEQUENTIAL if overlapping else MODE_PARALLEL), (kind, mode)


@pytest.mark.parametrize("kind,overlapping", KINDS, ids=[k for k, _ in KINDS])
def test_overlapping_descriptors_hostsim(hostsim_lib, oracle_lib, kind, overlapping):
    _check(hostsim_lib, oracle_lib, kind, overlapping)


@pytest.mark.gpu
@pytest.mark.parametrize("kind,overlapping", KINDS, ids=[k for k, _ in KINDS])
def test_overlapping_descriptors_gpu(gpu_lib, oracle_lib, kind, overlapping):
    _check(gpu_lib, oracle_lib, kind, overlapping)
