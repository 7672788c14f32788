"""Shared helpers: run the same program/maps/packets through two emulator libraries and compare.

`a` is the implementation under test (HIP product, or the host simulation on CPU); `b` is the
oracle (oracle/liboracle.so). Everything observable is compared bit for bit: per-packet status,
error code, pc, R0 kind/value, R0..R9 parity records, packet bytes written, final map state.
"""
from __future__ import annotations

import numpy as np

from gobpfld_amd import workloads as W
from gobpfld_amd.emulator import VM, MapDef, Settings


def setup_one(lib, program, maps, settings=None, entries=None):
    """A VM with `maps` (+ `entries`) and `program` (or a list: entrypoint first, tail-call targets after)."""
    vm = VM(settings or Settings(), lib=lib)
    idx = []
    for i, (mdef, init) in enumerate(maps):
        m = vm.add_map(mdef, init)
        idx.append(m)
        if entries and i in entries:
            for k, v in entries[i]:
                if k is None:
                    vm.map_push(m, v)  # QUEUE / STACK element
                else:
                    vm.map_update(m, k, v)
    # `program` may be a list of programs: the first is the entrypoint (tail-call targets follow)
    progs = program if program and isinstance(program[0], list) else [program]
    p = [vm.add_raw_program(x) for x in progs][0]
    vm.set_entrypoint(p)
    return vm, idx


def run_one(lib, program, maps, umem, descs, settings=None, regs=True, entries=None):
    vm, idx = setup_one(lib, program, maps, settings, entries)
    mem = umem.copy()
    r = vm.run_batch(mem, descs, want_regs=regs)
    dumps = [_dump(vm, m) for m in idx]
    vm.close()
    return r, dumps, mem


def kernel_sources(lib, cases) -> list[str]:
    """Sources of the per-program kernels of many cases (gobpfld_amd/aot.py sources: (program, maps,
    entries, settings) tuples or VM setup functions); cases that run on the interpreter contribute none."""
    from gobpfld_amd import aot
    return aot.sources(cases, lib=lib)


def precompile(lib, cases) -> int:
    """Build the per-program kernels of `cases` into the session's kernel cache now (worker processes,
    gobpfld_amd/kcache.py): the tests that run the cases one by one then load them. Returns the number of
    distinct kernels."""
    import tempfile
    from gobpfld_amd import kcache
    if not lib.has("set_kernel_cache"):
        return 0
    d = getattr(precompile, "dir", None) or tempfile.mkdtemp(prefix="xe-kernels-")
    precompile.dir = kcache.enable(lib, d)
    uniq = kernel_sources(lib, cases)
    kcache.fill(uniq, d)
    return len(uniq)


def _dump(vm, m):
    """Final state of map m: ARRAY raw bytes, HASH (keys, values), LRU_HASH (keys, values) + UsageList,
    QUEUE / STACK / PERF list of records."""
    from gobpfld_amd.emulator import MAP_LRU_HASH, MAP_LRU_PERCPU_HASH
    d = vm.map_dump(m)
    if vm.map_defs[m].type in (MAP_LRU_HASH, MAP_LRU_PERCPU_HASH):
        return {"entries_keys": d[0], "entries_values": d[1], "usage": vm.map_lru_order(m)}
    return d


def assert_same(a, b, what=""):
    ra, da, ma = a
    rb, db, mb = b
    bad = np.nonzero(ra.results != rb.results)[0]
    if len(bad):
        i = bad[0]
        raise AssertionError(f"{what}: result mismatch at packet {i}: got {ra.results[i]} want {rb.results[i]} "
                             f"({len(bad)} packets differ)")
    if ra.regs is not None and rb.regs is not None:
        badr = np.nonzero(ra.regs != rb.regs)[0]
        if len(badr):
            i = badr[0]
            raise AssertionError(f"{what}: register record mismatch at packet {i}: got {ra.regs[i]} want {rb.regs[i]}")
    assert (ra.verdicts == rb.verdicts).all(), f"{what}: verdicts differ"
    assert np.array_equal(ma, mb), f"{what}: packet bytes differ"
    for j, (x, y) in enumerate(zip(da, db)):
        if isinstance(x, (bytes, list)):
            assert x == y, f"{what}: map {j + 1} differs"
        elif isinstance(x, dict):
            assert x.keys() == y.keys()
            for k in x:
                assert np.array_equal(x[k], y[k]) if isinstance(x[k], np.ndarray) else x[k] == y[k], f"{what}: map {j + 1} {k} differs"
        else:
            assert len(x[0]) == len(y[0]), f"{what}: hash map {j + 1} entry count {len(x[0])} vs {len(y[0])}"
            assert np.array_equal(x[0], y[0]) and np.array_equal(x[1], y[1]), f"{what}: hash map {j + 1} differs"
    assert ra.stats["steps"] == rb.stats["steps"], f"{what}: steps {ra.stats['steps']} vs {rb.stats['steps']}"


def config_case(name: str, n: int, flows_cap: int | None = None):
    """(program, maps, entries, umem, descs) for a BASELINE config at reduced size."""
    prog = W.CONFIGS[name]["program"]()
    maps, entries = [], {}
    for i, (mdef, ents) in enumerate(W.workload_maps(name)):
        maps.append((mdef, None))
        if ents is not None:
            keys, vals = ents
            if flows_cap:
                keys, vals = keys[:flows_cap], vals[:flows_cap]
            entries[i] = [(k.tobytes(), v.tobytes()) for k, v in zip(keys, vals)]
    umem, descs = W.build_batch(name, 0, n)
    return prog, maps, entries, umem, descs


def packets(n: int, size: int = 64, seed: int = 1, fill=None):
    """n random packets of `size` bytes, back to back."""
    from gobpfld_amd._native import np_dtypes
    d_desc, _, _ = np_dtypes()
    rng = np.random.default_rng(seed)
    umem = rng.integers(0, 256, size=n * size, dtype=np.uint8) if fill is None else np.full(n * size, fill, np.uint8)
    descs = np.zeros(n, dtype=d_desc)
    descs["addr"] = np.arange(n) * size
    descs["len"] = size
    return umem, descs
