#!/usr/bin/env python3
"""Average per-dispatch counter values of the emulator kernels in rocprofv3 counter CSVs."""
import csv
import sys
from collections import defaultdict

agg = defaultdict(list)
meta = {}
for f in sys.argv[1:]:
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if not k.startswith("xe_"):
            continue
        agg[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
        meta[k] = {x: r[x] for x in ("Grid_Size", "Workgroup_Size", "LDS_Block_Size", "Scratch_Size", "VGPR_Count", "SGPR_Count")}
for k, m in meta.items():
    print(k, m)
for (k, c), v in sorted(agg.items()):
    print(f"{k:24s} {c:24s} n={len(v):3d} avg={sum(v) / len(v):.6g}")
