"""The scalar one-lane replay (xe_jit.cpp XE_JV_SEQ, xe_interp.h XE_UNIFORM; DESIGN §2 "The one-lane
replay"). An in-order replay of at least 16,384 packets on the per-program engine runs on a variant of
the kernel in which every lane of the one wave runs the same packet with the same state: loads are read
back wave-uniform, the arithmetic and branches that follow are scalar instructions, and each atomic is
issued by lane 0 alone. The reference's order is the Go harness's packet loop (emulator/vm.go:110-173).
Device == oracle on results, R0-R9 records, verdicts, map state and steps, for every config program
that has the fields lane model (the general model keeps its lane state in an arena and replays on the
plain kernel)."""
import pytest

from gobpfld_amd.emulator import MODE_SEQUENTIAL, Settings
from parity import assert_same, config_case, run_one

N = 20000  # > 16,384: the scalar variant's threshold (xe_runtime.cpp kSeqScalarMin)
# (c4: the rule-chain dispatch, xe_jit.cpp rule_chain_at, in the scalar form: its table reads are uniform)
CASES = {"c2": None, "c2rmw": None, "c3": 8192, "c3learn": 8192, "c3lru": 8192, "c4": None, "c5": 8192, "bpf2bpf": None}


def cases():
    """(program, maps, entries, settings) of the configs as this test runs them (tests/kernel_cases.py)."""
    out = []
    for name, cap in sorted(CASES.items()):
        prog, maps, entries, _, _ = config_case(name, 16, cap)
        out.append((prog, maps, entries, Settings(mode=MODE_SEQUENTIAL, engine=2)))
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(CASES))
def test_scalar_replay_equals_oracle(gpu_lib, oracle_lib, name):
    prog, maps, entries, umem, descs = config_case(name, N, CASES[name])
    s = Settings(mode=MODE_SEQUENTIAL, engine=2)
    a = run_one(gpu_lib, prog, maps, umem, descs, settings=s, entries=entries)
    b = run_one(oracle_lib, prog, maps, umem, descs, settings=Settings(mode=MODE_SEQUENTIAL), entries=entries)
    assert a[0].stats["mode_used"] == MODE_SEQUENTIAL
    assert_same(a, b, f"{name} scalar replay")
