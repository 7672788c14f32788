"""Differential fuzzing of the ordered maps (tests/fuzz.py gen_ordered_program): LRU_HASH lookups,
updates (pointer and IMM values, full starting maps: evictions), deletes and value writes, QUEUE / STACK
pushes, pops and peeks, PERF_EVENT_ARRAY outputs, beside a HASH map. Each program runs a stream of two
batches on one VM, so the second batch starts from the state the first left (stamps, order logs, keyed
hints, list heads). The implementation under test (host simulation of the device logic on CPU, the
MI355X with -m gpu) must equal the oracle's sequential VM on every observable after every batch:
results, R0-R9 records, verdicts, LRU entries and UsageList, list contents in order, steps.

Reference: emulator/vm.go:110-173 (packet order), maps_hash_lru.go:51-183, maps_queue.go:60-91,
maps_stack.go:60-90, maps_perf_event_array.go:101-115, helper_functions.go:76-374."""
import numpy as np
import pytest

from fuzz import gen_ordered_program, ordered_packets
from parity import _dump, assert_same, setup_one

N_PROGRAMS = 200


def run_stream(lib, prog, maps, entries, settings, batches):
    vm, idx = setup_one(lib, prog, maps, settings, entries)
    out = []
    for umem, descs in batches:
        mem = umem.copy()
        r = vm.run_batch(mem, descs, want_regs=True)
        out.append(((r, [_dump(vm, m) for m in idx], mem), r.stats["mode_used"]))
    vm.close()
    return out


def _batches(seed, n):
    return [ordered_packets(seed, n), ordered_packets(seed + 7777, n)]


def check_seed(lib, oracle_lib, seed, n, engine=None):
    prog, maps, entries, settings = gen_ordered_program(seed)
    if engine is not None:
        settings.engine = engine
    batches = _batches(seed, n)
    got = run_stream(lib, prog, maps, entries, settings, batches)
    want = run_stream(oracle_lib, prog, maps, entries, settings, batches)
    modes = []
    for b, ((ga, gm), (wa, _)) in enumerate(zip(got, want)):
        assert_same(ga, wa, f"ordered fuzz seed {seed} batch {b}")
        modes.append(gm)
    return modes


@pytest.mark.parametrize("block", range(4))
def test_ordered_fuzz_hostsim_equals_oracle(hostsim_lib, oracle_lib, block):
    per = N_PROGRAMS // 4
    modes = []
    for seed in range(block * per, (block + 1) * per):
        modes += check_seed(hostsim_lib, oracle_lib, seed, 96)
    # the generator must reach the parallel, keyed and in-order paths
    assert len(set(modes)) >= 2, modes


def test_ordered_fuzz_reaches_the_paths(hostsim_lib, oracle_lib):
    """Over the first programs the decisions are spread: parallel, keyed and in-order batches occur."""
    from gobpfld_amd.emulator import MODE_KEYED, MODE_PARALLEL, MODE_SEQUENTIAL
    modes = []
    for seed in range(40):
        modes += check_seed(hostsim_lib, oracle_lib, seed, 64)
    for m in (MODE_PARALLEL, MODE_KEYED, MODE_SEQUENTIAL):
        assert m in modes, (m, sorted(set(modes)))


@pytest.mark.gpu
def test_ordered_fuzz_device_interp(gpu_lib, oracle_lib):
    """All N_PROGRAMS on the device's interpreter engine (every mode decision, no per-program compile)."""
    from gobpfld_amd.emulator import ENGINE_INTERP
    for seed in range(N_PROGRAMS):
        check_seed(gpu_lib, oracle_lib, seed, 128, ENGINE_INTERP)


# the per-program kernels of these programs take the dynamic block form over the general lane model with
# every ordered-map helper compiled in: several CPU-minutes of hiprtc each, so the JIT leg keeps three
# (built ahead of time: gobpfld_amd/aot.py via tests/kernel_cases.py); the interpreter leg runs all
JIT_SEEDS = (25, 75, 100)  # (programs without a keyed variant: the keyed ones compile for up to 20 min)


@pytest.mark.gpu
def test_ordered_fuzz_device_jit(gpu_lib, oracle_lib):
    """Three of the programs on the per-program kernels (the same handlers, specialised per program)."""
    from gobpfld_amd.emulator import ENGINE_JIT
    for seed in JIT_SEEDS:
        check_seed(gpu_lib, oracle_lib, seed, 128, ENGINE_JIT)
