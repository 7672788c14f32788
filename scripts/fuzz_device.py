"""Round 6: the differential fuzzer (tests/fuzz.py gen_program: ALU / jumps / memory / HASH and ARRAY maps)
over more programs than the -m gpu suite runs, on the device's interpreter engine (no per-program
compile), each equal to the oracle on every observable (tests/parity.py assert_same).

    python scripts/fuzz_device.py FIRST LAST
"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

from gobpfld_amd import _native as N  # noqa: E402
from gobpfld_amd.emulator import ENGINE_INTERP  # noqa: E402
from fuzz import gen_program  # noqa: E402
from parity import assert_same, run_one  # noqa: E402
from test_fuzz_cpu import fuzz_packets  # noqa: E402


def main():
    lo, hi = int(sys.argv[1]), int(sys.argv[2])
    gpu = N.Lib(N.product_path(), "xe_")
    orc = N.Lib(ROOT / "oracle" / "liboracle.so", "orc_")
    bad = []
    for seed in range(lo, hi):
        prog, maps, entries, settings = gen_program(seed, 24 + seed % 64)
        umem, descs = fuzz_packets(seed, 64)
        settings.engine = ENGINE_INTERP
        try:
            assert_same(run_one(gpu, prog, maps, umem, descs, entries=entries, settings=settings),
                        run_one(orc, prog, maps, umem, descs, entries=entries, settings=settings), f"seed {seed}")
        except AssertionError as e:
            bad.append(seed)
            print("FAIL", seed, str(e)[:300], flush=True)
        if (seed - lo) % 250 == 0:
            print("seed", seed, "failures", len(bad), flush=True)
    print("programs", hi - lo, "failures", len(bad), bad[:10], flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
