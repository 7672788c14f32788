"""Ahead-of-time builds of per-program kernels, on a machine without a GPU.

A VM's per-program gfx950 kernel is generated from its programs and map geometry and compiled with
hiprtc (xe_jit.cpp), about 5-20 s of one CPU core each. A caller that knows its programs ahead of time
(a server's XDP programs, this repository's benchmark and test suite) builds them here, in worker
processes, into a kernel cache directory (include/xdpemu.h xe_set_kernel_cache); the VMs then load the
code objects instead of compiling. Code objects are named by a hash of the generated source, the
interpreter headers, the compile options and the target, so a stale object can never load: a changed
program, geometry or header simply misses and is compiled on first use as before.

The sources come from the host build of the runtime (tests/hostsim/libxdpemu_hostsim.so: the same
xe_runtime.cpp / xe_jit.cpp generator compiled with g++, which sets VMs up exactly as the device build
does and returns xe_kernel_source without touching a GPU); the compiles go through the product
library's xe_compile_kernel_source (hiprtc only, no device).

    python -m gobpfld_amd.aot                 # the benchmark configs and the -m gpu suite's kernels
    python -m gobpfld_amd.aot --bench-only    # bench.py / smoke() only (what build() does)
"""
from __future__ import annotations

import os
import sys
from pathlib import Path

from . import _native as N

ROOT = Path(__file__).resolve().parent.parent
KERNEL_DIR = ROOT / "gobpfld_amd" / "kernels"  # in-tree: travels with the library (git-ignored)
HOST_LIB = ROOT / "tests" / "hostsim" / "libxdpemu_hostsim.so"


def host_lib() -> N.Lib:
    return N.Lib(HOST_LIB, "xe_")


def sources(cases, lib: N.Lib | None = None, variants=(0, 1, 2)) -> list[str]:
    """Kernel sources (xe_kernel_source `variants`) of VMs set up from `cases`: callables taking a VM
    (setup functions) or (program, maps, entries, settings) tuples as the test suite lists them."""
    from .emulator import VM, EmulatorError, Settings
    lib = lib or host_lib()
    out = []
    for case in cases:
        vm = VM(case[3] if not callable(case) and case[3] else Settings(), lib=lib)
        try:
            if callable(case):
                case(vm)
            else:
                program, maps, entries, _ = case
                for i, (mdef, init) in enumerate(maps):
                    m = vm.add_map(mdef, init)
                    for k, v in (entries or {}).get(i, []):
                        if k is None:
                            vm.map_push(m, v)
                        else:
                            vm.map_update(m, k, v)
                progs = program if program and isinstance(program[0], list) else [program]
                vm.set_entrypoint([vm.add_raw_program(x) for x in progs][0])
            out += vm.kernel_sources(variants)
        except EmulatorError:
            continue  # a case the emulator refuses (it is tested for that) has no kernel
        finally:
            vm.close()
    return list(dict.fromkeys(out))


def bench_cases() -> list:
    """The VMs bench.py and smoke() set up (full-size maps: their geometry is part of the kernel)."""
    from . import workloads as W
    return [(lambda vm, n=name: W.setup_vm(vm, n))
            for name in ("c1", "c2", "c2rmw", "c3", "c3learn", "c3lru", "c3lrufull", "c4", "c5", "bpf2bpf")]


def test_sources() -> list[str]:
    """The -m gpu suite's kernels (tests/kernel_cases.py): every case's kernel and keyed variant, the
    verdict-only variant of the cases run without records."""
    tests = str(ROOT / "tests")
    if tests not in sys.path:
        sys.path.insert(0, tests)
    from kernel_cases import gpu_cases, gpu_lean_cases, gpu_seq_cases
    return (sources(gpu_cases(), variants=(0, 1)) + sources(gpu_lean_cases(), variants=(2,)) +
            sources(gpu_seq_cases(), variants=(3,)))


def build(srcs: list[str], cache_dir: str | os.PathLike = KERNEL_DIR, workers: int | None = None,
          prune: bool = False) -> dict:
    """Compile the kernel sources `srcs` the cache does not hold yet. prune: remove the code objects
    no source needs any more (the directory then holds exactly this set)."""
    from . import kcache
    d = Path(cache_dir)
    d.mkdir(parents=True, exist_ok=True)
    srcs = list(dict.fromkeys(srcs))
    errors = kcache.fill(srcs, d, workers=workers)
    slow = sorted(kcache.last_times, key=lambda x: -x[0])[:5]
    for t, src in slow:  # the kernels that dominate a cold build (what made them slow: their #defines)
        if t > 60:
            print(f"aot: {t:.0f} s  " + " ".join(l.split()[1] + "=" + (l.split() + ["", ""])[2]
                                                  for l in src.splitlines()[:14] if l.startswith("#define")), file=sys.stderr)
    removed = 0
    if prune:
        keep = {kcache.code_object_name(s) for s in srcs}
        for f in d.glob("xe_*.co"):
            if f.name not in keep:
                f.unlink()
                removed += 1
    return {"kernels": len(srcs), "errors": errors, "pruned": removed, "dir": str(d)}


def build_all(workers: int | None = None, tests: bool = True) -> dict:
    """The benchmark / smoke kernels, and with `tests` the -m gpu suite's (then stale objects are pruned)."""
    # (variant 3: the scalar one-lane replay of the ordered-path lines)
    return build(sources(bench_cases(), variants=(0, 1, 2, 3)) + (test_sources() if tests else []), KERNEL_DIR,
                 workers=workers, prune=tests)


if __name__ == "__main__":
    r = build_all(tests="--bench-only" not in sys.argv)
    print(f"{r['kernels']} kernels in {r['dir']} ({len(r['errors'])} failed, {r['pruned']} stale removed)")
    for e in r["errors"][:5]:
        print(e[:500])
