"""The per-program kernels the -m gpu suite builds, listed once so a session can build them all up front
in worker processes (gobpfld_amd/kcache.py) while the first tests run; each test's own build then finds
its kernel in the cache (or compiles it itself if it is not there yet: the cache only saves time)."""
from __future__ import annotations

from gobpfld_amd.emulator import MAP_ARRAY, MAP_HASH, MapDef, Settings

JIT = 2


def gpu_cases():
    """(program, maps, entries, settings) — or a function setting a VM up — in roughly the order the
    suite reaches them."""
    from fuzz import gen_program
    from kats import KATS
    from parity import config_case
    cases = []
    for name, cap in (("c1", None), ("c2", None), ("c3", 8192), ("c4", None), ("c5", 8192), ("bpf2bpf", None)):
        prog, maps, entries, _, _ = config_case(name, 16, cap)
        cases.append((prog, maps, entries, Settings(engine=JIT)))
    cases += [(k["program"], k["maps"], k["entries"], Settings(engine=JIT)) for k in KATS]
    for seed in range(48):
        prog, maps, entries, settings = gen_program(seed, 24 + seed % 64)
        settings.engine = JIT
        cases.append((prog, maps, entries, settings))
    import test_keyed as K
    for c in sorted(K.CASES):
        cases.append((*K.CASES[c](), Settings(engine=JIT)))
    prog, maps, entries, _, _ = config_case("c3learn", 16)
    cases.append((prog, maps, entries, Settings(engine=JIT)))
    cases.append((K.prog_escape(), [(MapDef(MAP_HASH, 4, 8, 64), None), (MapDef(MAP_ARRAY, 4, 8, 8), None)], None,
                  Settings(engine=JIT)))
    cases.append((K.prog_many_keys(), [(MapDef(MAP_ARRAY, 4, 8, 16384), None)], None, Settings()))
    cases.append((K.prog_learn_in_call(), [(MapDef(MAP_HASH, 4, 8, 64), None)], None, Settings()))
    cases.append((K.prog_first_seen(), [(MapDef(MAP_HASH, 4, 8, 256), None)], None, Settings()))
    # the shard-exchange programs (tests/test_multirank.py, test_gpu_multi.py) and the LRU golden program
    import test_lru_golden as G
    import test_multirank as M
    for name, _, cap, _ in M.CASES:
        cases.append(lambda vm, name=name, cap=cap: M._setup(vm, name, cap))
    cases.append(lambda vm: vm.set_entrypoint(vm.add_raw_program(G._program(G._map(vm)))))
    import test_ordered_par as O
    for name, (build, _, entries, _) in O.CASES.items():
        cases.append((build(), O.case_maps(name), entries, Settings()))
    import test_rule_chain as RC
    for kind in RC.KINDS:
        cases.append((RC.prog_rules(kind), [], None, Settings(engine=JIT)))
    for seed in RC.RANDOM_SEEDS:
        cases.append((RC.prog_random(seed), [], None, Settings(engine=JIT)))
    import test_segments as SG
    for name in SG.CASES:
        prog, maps, entries = SG._case(name)
        cases.append((prog, maps, entries, Settings()))
    from gobpfld_amd import workloads as W
    cases.append(lambda vm: W.setup_vm(vm, "c3lru"))
    import test_ref_examples as R
    for prog in (R.from_text(), R.from_literals()):
        cases.append((prog, [R.STATS_MAP], None, Settings(engine=JIT)))
    import test_key_shadow as KS
    cases += KS.kernel_cases()
    # LRU evictions (tests/test_lru_evict.py): the learning program on its preloaded maps, the IMM-value
    # update program, and every 8th ordered-map fuzz program (tests/test_fuzz_ordered.py)
    import test_lru_evict as LE
    cases.append(lambda vm: LE._vm_setup(vm, LE._program(), LE.MAX, LE.MAX))
    cases.append(lambda vm: LE._vm_setup(vm, LE._program(), LE.MAX, LE.MAX - 10))
    cases.append(lambda vm: LE._vm_setup(vm, LE._program(), LE.MAX, 0))
    cases.append(lambda vm: LE._vm_setup(vm, LE._program(), 5000, 5000))
    for mx, _, _, _ in LE.IMM_CASES.values():
        cases.append(lambda vm, mx=mx: LE._vm_setup(vm, LE._program_imm(), mx, mx))
    # hash maps above 4M entries (tests/test_large_map.py)
    import test_large_map as LM
    for size in ("3M", "16M", "32M", "128M"):
        cases.append((LM.prog_learn_u16(), [(MapDef(MAP_HASH, 4, 8, LM.SIZES[size]), None)], LM._entries(), Settings(engine=JIT)))
    cases.append((LM.prog_learn_u32(), [(MapDef(MAP_HASH, 4, 8, LM.LIVE_MAX), None)], None, Settings()))
    from fuzz import gen_ordered_program
    import test_fuzz_ordered as FO
    for seed in FO.JIT_SEEDS:
        prog, maps, entries, settings = gen_ordered_program(seed)
        settings.engine = JIT
        cases.append((prog, maps, entries, settings))
    return cases


def gpu_seq_cases():
    """The cases whose in-order replays reach the scalar replay variant (>= 16,384 packets on the
    per-program engine): its kernel (xe_jit.cpp XE_JV_SEQ)."""
    import test_seq_scalar as SS
    import test_lru_evict as LE
    import test_ordered_par as O
    cases = SS.cases()
    cases.append(lambda vm: LE._vm_setup(vm, LE._program(), LE.MAX, LE.MAX))
    cases.append(lambda vm: LE._vm_setup(vm, LE._program(), LE.MAX, 0))
    for name, (build, _, entries, _) in O.CASES.items():
        cases.append((build(), O.case_maps(name), entries, Settings()))
    from gobpfld_amd import workloads as W
    cases.append(lambda vm: W.setup_vm(vm, "c3lru"))
    return cases


def gpu_lean_cases():
    """The cases the suite also runs without result records (device-resident batches with verdicts only):
    their verdict-only kernel variant. The full-size config tests share bench.py's geometry (its kernels
    come with the benchmark's)."""
    from parity import config_case
    cases = []
    for name, cap in (("c2", None), ("c5", 8192)):
        prog, maps, entries, _, _ = config_case(name, 16, cap)
        cases.append((prog, maps, entries, Settings()))
    import test_lru_golden as G
    import test_multirank as M
    for name, _, cap, _ in M.CASES:
        cases.append(lambda vm, name=name, cap=cap: M._setup(vm, name, cap))
    cases.append(lambda vm: vm.set_entrypoint(vm.add_raw_program(G._program(G._map(vm)))))
    import test_wave_steps as WS
    cases.append(WS.setup_errors)
    import test_rule_chain as RC
    for kind in RC.KINDS:
        cases.append((RC.prog_rules(kind), [], None, Settings(engine=JIT)))
    return cases
