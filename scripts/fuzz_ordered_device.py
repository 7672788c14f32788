"""Round 6: the ordered-map fuzzer (tests/fuzz.py gen_ordered_program) over more programs than the -m gpu
suite runs, on the device's interpreter engine (no per-program compile), two batches per program, each
equal to the oracle's single VM. Prints the mode counts and any failing seed.

    python scripts/fuzz_ordered_device.py FIRST LAST PACKETS
"""
import collections
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

from gobpfld_amd import _native as N  # noqa: E402
from gobpfld_amd.emulator import ENGINE_INTERP  # noqa: E402
import test_fuzz_ordered as F  # noqa: E402


def main():
    lo, hi, n = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    gpu = N.Lib(N.product_path(), "xe_")
    orc = N.Lib(ROOT / "oracle" / "liboracle.so", "orc_")
    modes, bad = collections.Counter(), []
    for s in range(lo, hi):
        try:
            for m in F.check_seed(gpu, orc, s, n, ENGINE_INTERP):
                modes[m] += 1
        except AssertionError as e:
            bad.append((s, str(e)[:300]))
            print("FAIL", s, str(e)[:300], flush=True)
        if (s - lo) % 100 == 0:
            print("seed", s, dict(modes), flush=True)
    print("modes", dict(modes), "failures", len(bad), bad[:3], flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
