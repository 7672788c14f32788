"""Round 6: the differential fuzzer (tests/fuzz.py gen_program) on the per-program kernels (the product's
hot path) over more programs than the -m gpu suite's 48, each equal to the oracle on every observable.
Build their kernels ahead of time here first (no GPU), into the in-tree cache the product loads:

    python scripts/fuzz_jit_device.py --aot FIRST LAST     # CPU: hiprtc in worker processes
    python scripts/fuzz_jit_device.py FIRST LAST           # GPU
"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

from gobpfld_amd import _native as N  # noqa: E402
from gobpfld_amd.emulator import ENGINE_JIT  # noqa: E402
from fuzz import gen_program  # noqa: E402
from parity import assert_same, run_one  # noqa: E402
from test_fuzz_cpu import fuzz_packets  # noqa: E402


def case(seed):
    prog, maps, entries, settings = gen_program(seed, 24 + seed % 64)
    settings.engine = ENGINE_JIT
    return prog, maps, entries, settings


def main():
    if sys.argv[1] == "--aot":
        from gobpfld_amd import aot
        lo, hi = int(sys.argv[2]), int(sys.argv[3])
        r = aot.build(aot.sources([case(s) for s in range(lo, hi)], variants=(0,)), prune=False)
        print(r["kernels"], "kernels,", len(r["errors"]), "failed")
        return
    lo, hi = int(sys.argv[1]), int(sys.argv[2])
    gpu = N.product()  # (with the in-tree kernel cache)
    orc = N.Lib(ROOT / "oracle" / "liboracle.so", "orc_")
    bad, jit = [], 0
    for seed in range(lo, hi):
        prog, maps, entries, settings = case(seed)
        umem, descs = fuzz_packets(seed, 64)
        try:
            a = run_one(gpu, prog, maps, umem, descs, entries=entries, settings=settings)
            assert_same(a, run_one(orc, prog, maps, umem, descs, entries=entries, settings=settings), f"seed {seed}")
            jit += a[0].stats["engine_used"] == ENGINE_JIT
        except AssertionError as e:
            bad.append(seed)
            print("FAIL", seed, str(e)[:300], flush=True)
        if (seed - lo) % 25 == 0:
            print("seed", seed, "failures", len(bad), flush=True)
    print("programs", hi - lo, "on the per-program kernels", jit, "failures", len(bad), bad[:10], flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
