#!/usr/bin/env python3
"""HBM traffic per launch of the emulator kernel from PMC passes (scripts/gpu_r3_pmc.sh,
scripts/gpu_r4_configs.sh: separate rocprofv3 --pmc runs of FETCH_SIZE, WRITE_SIZE and
TCC_EA0_RDREQ_sum + TCC_EA0_ATOMIC_sum over `bench.py --config <c> --steps 5`).

  python scripts/traffic.py <pmc dir (gpurun_out/r4cfg)> <out dir (profiles/r4)> [configs: c2 c3 c4 c4f c5]

Correction as MI355X_MICROARCH.md prescribes (HBM/rocprofv3 section): on gfx950 FETCH_SIZE reports half
of the bytes of wide coalesced streaming reads, so `hbm_bytes_per_launch` = 2 x FETCH_SIZE + WRITE_SIZE.
That is exact for the streaming parts (descriptors, back-to-back header windows) and an upper bound for
the random 64-B hash probe groups, which the round-2 calibration (tools/calib_fetch*.hip,
profiles/r2/fetch_size_calibration*.json) found counted at x1; `bounds_x1_x2` gives both ends.
"""
import collections
import csv
import glob
import json
import sys
from pathlib import Path

PKTS = {"c2": 16777216, "c3": 16777216, "c4": 16777216, "c4f": 16777216, "c5": 33554432}


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


def main() -> None:
    src, dst = Path(sys.argv[1]), Path(sys.argv[2])
    dst.mkdir(parents=True, exist_ok=True)
    names = sys.argv[3:] or list(PKTS)
    for name in names:
        n = PKTS[name]
        fetch = per_launch(src / f"{name}_fetch")["FETCH_SIZE"] * 1024
        write = per_launch(src / f"{name}_write")["WRITE_SIZE"] * 1024
        rq = per_launch(src / f"{name}_rdreq")
        alg = 84 * n
        hbm = 2 * fetch + write
        d = {
            "workload": name, "packets": n, "kernel": "xe_jit_kernel", "dispatches": rq["dispatches"],
            "fetch_size_bytes_raw": round(fetch), "write_size_bytes": round(write),
            "tcc_ea0_rdreq": round(rq["TCC_EA0_RDREQ_sum"]), "tcc_ea0_atomic": round(rq["TCC_EA0_ATOMIC_sum"]),
            "per_packet": {"fetch_raw": round(fetch / n, 1), "write": round(write / n, 1),
                           "rdreq": round(rq["TCC_EA0_RDREQ_sum"] / n, 3),
                           "memory_side_atomics": round(rq["TCC_EA0_ATOMIC_sum"] / n, 3)},
            "hbm_bytes_per_launch": round(hbm),
            "hbm_bytes_per_packet": round(hbm / n, 1),
            "bounds_x1_x2": [round(fetch + write), round(hbm)],
            "alg_bytes_per_launch": alg,
            "traffic_over_alg": round(hbm / alg, 3),
            "correction": "2 x FETCH_SIZE + WRITE_SIZE (MI355X_MICROARCH.md: FETCH_SIZE reports half of wide streaming reads)",
            "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE / TCC_EA0_RDREQ_sum,TCC_EA0_ATOMIC_sum, separate passes of "
                      f"python3 bench.py --config {name} --packets {n} --steps 5 --warmup 1 ({src})",
        }
        # the round-2 shape calibration (profiles/r2/fetch_size_calibration*.json): streaming parts x2,
        # random probe groups x1, 1500-B-stride windows counted at 0.82 of the 64-B blocks they touch
        if name in ("c2", "c5"):
            cal = fetch + 40 * n  # descriptors + back-to-back windows stream (counted half); probes x1
        elif name == "c4":
            cal = 16 * n + (fetch - 8 * n) / (385.0e6 / 469.8e6)
        elif name == "c4f":  # frame-aligned windows: one 64-B block per 2-KiB frame (x1, one request each)
            cal = fetch + 8 * n  # + the descriptors' streaming half
        else:
            cal = fetch + 8 * n  # IMIX: descriptors stream; windows and probes at x1 (a lower bound)
        d["calibrated_estimate"] = {"hbm_bytes_per_packet": round((cal + write) / n, 1),
                                    "traffic_over_alg": round((cal + write) / alg, 3),
                                    "model": "round-2 per-shape calibration of FETCH_SIZE (profiles/r2/fetch_size_calibration*.json, applied by scripts/traffic.py main)"}
        (dst / f"{name}_traffic.json").write_text(json.dumps(d, indent=1) + "\n")
        print(name, "calibrated", d["calibrated_estimate"])
        print(name, d["per_packet"], "hbm/pkt", d["hbm_bytes_per_packet"], "ratio", d["traffic_over_alg"])


if __name__ == "__main__":
    main()
