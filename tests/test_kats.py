"""Known-answer tests (tests/kats.py) on the CPU: the oracle reproduces each quirk's answer read off
the cited reference line, and the host simulation of the device logic equals the oracle."""
import pytest

from kats import KATS
from parity import assert_same, packets, run_one


def _run(lib, k):
    umem, descs = packets(4, k["pkt"], seed=7)
    return run_one(lib, k["program"], k["maps"], umem, descs, entries=k["entries"])


@pytest.mark.parametrize("k", KATS, ids=[k["name"] for k in KATS])
def test_oracle_known_answer(oracle_lib, k):
    res, _, _ = _run(oracle_lib, k)
    r = res.results[0]
    want = k["expect"]
    if want is None:
        return
    status, val = want
    assert r["status"] == status, f"{k['name']} ({k['cite']}): status {r['status']} code {r['code']} want {status}"
    if val is None:
        return
    if status == 0:
        assert r["r0"] == val, f"{k['name']} ({k['cite']}): r0 {r['r0']:#x} want {val:#x}"
    else:
        assert r["code"] == val, f"{k['name']} ({k['cite']}): code {r['code']} want {val}"


@pytest.mark.parametrize("k", KATS, ids=[k["name"] for k in KATS])
def test_hostsim_equals_oracle(oracle_lib, hostsim_lib, k):
    assert_same(_run(hostsim_lib, k), _run(oracle_lib, k), k["name"])
