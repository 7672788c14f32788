#!/usr/bin/env python3
"""Per-pass device time of keyed ordered execution from a rocprofv3 kernel trace of
scripts/keyed_profile.py (one C3-learn batch per run): every dispatch of the last run in launch order
with its duration, and the sum per pass (SPEC = the first xe_jit_kernel of a run, the build steps, the
parallel pass of the packets on no chain, the chain pass).

usage: python scripts/keyed_passes.py <rocprofv3 -d DIR> [out.json]
"""
import csv
import glob
import json
import sys


def main() -> None:
    f = glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    # the last run: its three emulator launches are SPEC, the parallel pass and the chain pass
    last = rows[-80:]
    jit = [i for i, r in enumerate(last) if r["Kernel_Name"].startswith("xe_jit_kernel")]
    start = jit[-3] if len(jit) >= 3 else 0
    seq = last[start:]
    out, passes = [], {"spec": 0.0, "build": 0.0, "parallel": 0.0, "chains": 0.0, "other": 0.0}
    jit_seen = 0
    for r in seq:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        name = r["Kernel_Name"]
        if name.startswith("xe_jit_kernel"):
            key = ("spec", "parallel", "chains")[min(jit_seen, 2)]
            jit_seen += 1
        elif "keyed" in name or "Radix" in name or "Scan" in name or "radix" in name or "scan" in name:
            key = "build"
        else:
            key = "other"
        passes[key] += d
        out.append({"kernel": name[:60], "ms": round(d, 4), "pass": key})
    res = {"dispatches": out, "pass_ms": {k: round(v, 4) for k, v in passes.items()},
           "total_ms": round(sum(passes.values()), 4)}
    print(json.dumps(res["pass_ms"]), res["total_ms"])
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(json.dumps(res, indent=1) + "\n")


if __name__ == "__main__":
    main()
