#!/usr/bin/env python3
"""HBM bytes per launch of the emulator kernel from rocprofv3 FETCH_SIZE / WRITE_SIZE passes.

  python scripts/pmc_traffic.py <config> <packets> <fetch counter csv> <write counter csv> <out json>
FETCH_SIZE is doubled (gfx950 reports half of 16-B/lane streaming reads, MI355X_MICROARCH.md)."""
import csv
import json
import sys

name, n, fcsv, wcsv, out = sys.argv[1], int(sys.argv[2]), sys.argv[3], sys.argv[4], sys.argv[5]


def avg(f):
    v = [float(r["Counter_Value"]) for r in csv.DictReader(open(f)) if r["Kernel_Name"].startswith("xe_jit")]
    return sum(v) / len(v), len(v)


fk, nd = avg(fcsv)
wk, _ = avg(wcsv)
d = {"workload": name, "packets": n, "kernel": "xe_jit_kernel", "dispatches": nd, "fetch_size_kb_avg": fk,
     "write_size_kb_avg": wk, "hbm_bytes_per_launch": round(fk * 1024 * 2 + wk * 1024),
     "correction": "FETCH_SIZE x2 (gfx950 reports half of 16-B/lane streaming reads, MI355X_MICROARCH.md HBM "
                   "section); WRITE_SIZE as reported",
     "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes of python3 bench.py --steps 3 "
               "--warmup 1 --no-cpu-baseline"}
json.dump(d, open(out, "w"), indent=1)
print(d["hbm_bytes_per_launch"])
