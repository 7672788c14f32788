#!/usr/bin/env python3
"""Per-launch SQ counters of the emulator kernel (one rocprofv3 --pmc pass of 8 SQ counters over
`bench.py --config <c> --steps 3`) as profiles/<round>/<config>_sq_counters.json, in the form bench.py's
sq_issue() reads; for C4 also the lane utilisation of its block-structured form, computed on the CPU from
the oracle's per-packet step counts (a chunk's wave walks the blocks until its slowest lane is done).

  python scripts/sq_summary.py <pmc dir> <config> <packets> <out.json> [note]
"""
import collections
import csv
import glob
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def per_launch(d: Path) -> tuple[dict, int]:
    f = glob.glob(str(d / "**" / "*counter_collection.csv"), recursive=True)[0]
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        if r["Kernel_Name"].startswith("xe_jit_kernel"):
            acc[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    out = collections.defaultdict(float)
    for k in acc:
        for c, v in acc[k].items():
            out[c] += v / len(acc)
    return dict(out), len(acc)


def lane_utilisation(name: str, sample: int = 65536) -> dict:
    """Σ per-packet steps ÷ (64 x Σ over chunks of the chunk's longest packet): the share of the wave's
    emulated instruction slots that retire a lane's instruction (oracle step counts, first `sample` packets)."""
    import numpy as np
    from gobpfld_amd import _native as N
    from gobpfld_amd import workloads as W
    from gobpfld_amd.emulator import VM, Settings
    vm = VM(Settings(), lib=N.Lib(ROOT / "oracle" / "liboracle.so", "orc_"))
    W.setup_vm(vm, name)
    umem, descs = W.build_batch(name, 0, sample)
    r = vm.run_batch(umem, descs, want_regs=True)
    vm.close()
    steps = r.regs["steps"].astype(np.int64).reshape(-1, 64)
    return {"lane_steps": int(steps.sum()), "wave_steps": int(64 * steps.max(axis=1).sum()),
            "lane_utilisation": round(float(steps.sum() / (64 * steps.max(axis=1).sum())), 4),
            "sample_packets": sample, "mean_steps": round(float(steps.mean()), 2)}


def main() -> None:
    src, name, n, dst = Path(sys.argv[1]), sys.argv[2], int(sys.argv[3]), Path(sys.argv[4])
    note = sys.argv[5] if len(sys.argv) > 5 else ""
    pl, disp = per_launch(src)
    chunks = n / 64
    d = {"workload": name, "packets": n, "kernel": "xe_jit_kernel (verdict-only variant)", "dispatches": disp,
         "per_launch": pl, "per_64_packet_chunk": {k: round(v / chunks, 1) for k, v in pl.items()},
         "wait_any_frac_of_wave_cycles": round(pl["SQ_WAIT_ANY"] / max(1.0, pl["SQ_WAVE_CYCLES"]), 4),
         "source": f"rocprofv3 --pmc (8 SQ counters, one pass) -- python3 bench.py --config {name} --steps 3 ({src})",
         "note": "SQ_*_CYCLES counters are in units of 4 cycles on gfx9" + (f"; {note}" if note else "")}
    if name in ("c4", "c4f"):
        d["block_form"] = lane_utilisation(name)
    dst.write_text(json.dumps(d, indent=1) + "\n")
    print(json.dumps({k: d[k] for k in ("per_64_packet_chunk", "wait_any_frac_of_wave_cycles")}), d.get("block_form"))


if __name__ == "__main__":
    main()
