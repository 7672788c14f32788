#!/usr/bin/env python3
"""HBM traffic per launch for C2-C5 from the round-2 PMC passes, corrected per access shape.

  python scripts/traffic_final.py <pmc dir (gpurun_out/r2g10)> <out dir (profiles/r2/final)>

FETCH_SIZE counts TCC_EA0_RDREQ x 64 B. tools/calib_fetch.hip / calib_fetch2.hip measured what that
means per shape on gfx950 (profiles/r2/fetch_size_calibration*.json):
  * wide streaming reads (16 B per lane, consecutive lanes): half of the bytes (128-B requests tallied
    at 64 B) -> x2;
  * random 64-B blocks (the hash probe groups), in HBM or in the Infinity Cache: the bytes, x1;
  * 64-B header windows at a 1500-B stride (LDS-DMA from the 16-B aligned address below the packet):
    0.82 of the 64-B blocks they touch (adjacent halves of a 128-B line merge into one request).
So one factor does not fit a kernel that mixes the shapes. The corrected estimate adds back what the
counter misses of the parts whose bytes are known from the batch layout: the streaming descriptors
(and, for back-to-back 64-B packets, the header windows) count half; the 1500-B windows count 0.82 of
their touched blocks. Whatever FETCH_SIZE holds beyond those parts is taken at x1 (the probe groups).
WRITE_SIZE is exact for the verdict stores; memory-side atomics appear in it at 32 B per request.
"""
import collections
import csv
import glob
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from gobpfld_amd import workloads as W  # noqa: E402

PKTS = {"c2": 16777216, "c3": 16777216, "c4": 16777216, "c5": 33554432}
WIN1500_COUNTED = 385.0e6 / 469.8e6  # calib_fetch2 win1500: FETCH_SIZE bytes / touched 64-B block bytes


def per_launch(d: Path) -> dict:
    f = glob.glob(str(d / "**" / "*counter_collection.csv"), recursive=True)[0]
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        if r["Kernel_Name"].startswith("xe_jit_kernel"):
            acc[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    out = collections.defaultdict(float)
    for k in acc:
        for c, v in acc[k].items():
            out[c] += v / len(acc)
    return dict(out) | {"dispatches": len(acc)}


def touched_blocks(name: str, n: int) -> int:
    """64-B blocks the header windows touch: [a & ~15, (a & ~15) + min(64, len)) per packet."""
    sizes = W.packet_sizes(name, np.arange(n, dtype=np.uint64)).astype(np.int64)
    a = np.zeros(n, dtype=np.int64)
    a[1:] = np.cumsum(sizes[:-1])
    lo = a & ~15
    hi = lo + np.minimum(64, sizes + (a & 15)) - 1
    return int(((hi >> 6) - (lo >> 6) + 1).sum())


def main() -> None:
    src, dst = Path(sys.argv[1]), Path(sys.argv[2])
    dst.mkdir(parents=True, exist_ok=True)
    for name, n in PKTS.items():
        fetch = per_launch(src / f"{name}_fetch")["FETCH_SIZE"] * 1024
        write = per_launch(src / f"{name}_write")["WRITE_SIZE"] * 1024
        rq = per_launch(src / f"{name}_rdreq")
        alg = 84 * n
        if name in ("c2", "c5"):  # descriptors + back-to-back 64-B packets: one streaming read set
            stream = 80 * n
            fetched = fetch + stream / 2
            model = "descriptors + 64-B headers streaming (counted x0.5); the rest (C5: probe groups) x1"
        elif name == "c4":  # streaming descriptors, windows at the 1500-B stride
            fetched = 16 * n + (fetch - 8 * n) / WIN1500_COUNTED
            model = "descriptors streaming (x0.5); 1500-B-stride windows counted 0.82 of their touched blocks"
        else:  # C3 IMIX: descriptors streaming; windows and probes taken at x1 (a lower bound)
            fetched = fetch + 8 * n
            model = "descriptors streaming (x0.5); windows and probe groups at x1 (lower bound; x2 upper)"
        d = {
            "workload": name, "packets": n, "kernel": "xe_jit_kernel", "dispatches": rq["dispatches"],
            "fetch_size_bytes_raw": round(fetch), "write_size_bytes": round(write),
            "tcc_ea0_rdreq": round(rq["TCC_EA0_RDREQ_sum"]), "tcc_ea0_atomic": round(rq["TCC_EA0_ATOMIC_sum"]),
            "per_packet": {"fetch_raw": round(fetch / n, 1), "write": round(write / n, 1),
                           "rdreq": round(rq["TCC_EA0_RDREQ_sum"] / n, 3),
                           "memory_side_atomics": round(rq["TCC_EA0_ATOMIC_sum"] / n, 3)},
            "hbm_bytes_per_launch": round(fetched + write),
            "bounds_x1_x2": [round(fetch + write), round(2 * fetch + write)],
            "alg_bytes_per_launch": alg,
            "traffic_over_alg": round((fetched + write) / alg, 3),
            "model": model,
            "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE / TCC_EA0_RDREQ_sum,TCC_EA0_ATOMIC_sum, separate passes "
                      f"of python3 bench.py --config {name} --steps 5 --warmup 1 (scripts/r2_gpu10.sh)",
        }
        if name == "c3":
            d["header_window_blocks64_touched"] = touched_blocks(name, n)
        (dst / f"{name}_traffic.json").write_text(json.dumps(d, indent=1) + "\n")
        print(name, d["per_packet"], "hbm/pkt", round((fetched + write) / n, 1), "ratio", d["traffic_over_alg"])


if __name__ == "__main__":
    main()
