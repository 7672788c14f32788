#!/usr/bin/env python3
"""Summarise a gpurun_out/r2c counter run (scripts/r2_counters.sh) into profiles/r2/.

Per config: HBM bytes per launch of xe_jit_kernel from the FETCH_SIZE (x2, pinned by the calibration
below) and WRITE_SIZE passes, the ratio to the algorithmic bytes, memory-side atomic requests, the SQ
wait split and the kernel-trace average; the FETCH_SIZE calibration (1 GiB streamed through plain
16-B loads and through LDS-DMA); the C5 cost split (map adds compiled out) and the C3 per-process
kernel times.

  python scripts/r2_summarize.py gpurun_out/r2c profiles/r2
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

src, dst = sys.argv[1], sys.argv[2]
os.makedirs(dst, exist_ok=True)
PACKETS = {"c3": 16777216, "c4": 16777216, "c5": 33554432}
ALG = {"c3": 84, "c4": 84, "c5": 84}  # 16 desc + min(len, 64) + 4 verdict (every C3 packet is >= 64 B)


def counters(d, prefix="xe_jit"):
    acc = defaultdict(list)
    for f in glob.glob(os.path.join(src, d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Kernel_Name"].startswith(prefix):
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def bench_line(log):
    for line in open(os.path.join(src, log)):
        if line.startswith('{"metric"'):
            return json.loads(line)
    return None


cal = {}
for f in glob.glob(os.path.join(src, "calib", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        cal.setdefault(r["Kernel_Name"].split("(")[0], []).append(float(r["Counter_Value"]))
calib = {k: {"fetch_size_kb": sum(v) / len(v), "bytes_read": 1 << 30,
             "ratio_bytes_per_fetch_kb": (1 << 30) / (sum(v) / len(v) * 1024)} for k, v in cal.items() if k.startswith("stream")}
json.dump({"what": "1 GiB read once per launch (4x the 256 MiB Infinity Cache) through 16-B-per-lane plain loads "
                   "(stream_plain) and 16-B-per-lane LDS-DMA global_load_lds_dwordx4 (stream_lds), tools/calib_fetch.hip; "
                   "FETCH_SIZE reports half of the bytes on both paths, so the emulator's descriptor and header-window "
                   "reads are counted x2", "kernels": calib}, open(os.path.join(dst, "fetch_size_calibration.json"), "w"), indent=1)

summary = {}
for c in ("c3", "c4", "c5"):
    f = counters(f"{c}_fetch")["FETCH_SIZE"]
    w = counters(f"{c}_write")["WRITE_SIZE"]
    tcc = counters(f"{c}_tcc")
    sq = counters(f"{c}_sq")
    n = PACKETS[c]
    hbm = f * 1024 * 2 + w * 1024
    alg = n * ALG[c]
    kt = [r for r in csv.DictReader(open(os.path.join(src, f"{c}_kt", "run_kernel_stats.csv"))) if r["Name"] == "xe_jit_kernel"][0]
    b = bench_line(f"{c}_kt.log")
    atom = tcc.get("TCC_EA0_ATOMIC_sum", 0.0)
    d = {"workload": c, "packets": n, "kernel": "xe_jit_kernel", "fetch_size_kb_avg": f, "write_size_kb_avg": w,
         "hbm_bytes_per_launch": round(hbm), "alg_bytes_per_launch": alg, "traffic_over_alg": round(hbm / alg, 3),
         "fetch_bytes_per_packet": round(f * 2048 / n, 1), "write_bytes_per_packet": round(w * 1024 / n, 1),
         "tcc_ea0_atomic_per_launch": atom, "atomics_per_packet": round(atom / n, 3),
         "tcc_hit": tcc.get("TCC_HIT_sum"), "tcc_miss": tcc.get("TCC_MISS_sum"),
         "sq_wait_any_frac": round(sq["SQ_WAIT_ANY"] / sq["SQ_WAVE_CYCLES"], 3),
         "sq_wait_inst_any_frac": round(sq["SQ_WAIT_INST_ANY"] / sq["SQ_WAVE_CYCLES"], 3),
         "sq_active_inst_any_frac": round(sq["SQ_ACTIVE_INST_ANY"] / sq["SQ_WAVE_CYCLES"], 3),
         "sq_insts_valu_per_packet": round(sq["SQ_INSTS_VALU"] * 64 / n, 1),
         "kernel_trace_avg_ms": float(kt["AverageNs"]) / 1e6, "bench_avg_kernel_ms": b["roofline"]["avg_kernel_ms"] if b else None,
         "bench_kernel_ms_steps": b["roofline"].get("kernel_ms_steps") if b else None,
         "correction": "FETCH_SIZE x2 (profiles/r2/fetch_size_calibration.json); WRITE_SIZE as reported (map atomics "
                       "appear in it at 32 B per memory-side request)",
         "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE / TCC_EA0_ATOMIC_sum,TCC_HIT_sum,TCC_MISS_sum / SQ group, "
                   f"separate passes of python3 bench.py --config {c} --steps 5 --warmup 1 --no-cpu-baseline --no-e2e"}
    json.dump(d, open(os.path.join(dst, f"{c}_traffic.json"), "w"), indent=1)
    if b:
        json.dump(b, open(os.path.join(dst, f"bench_{c}_under_rocprof.json"), "w"))
    os.system(f"cp {os.path.join(src, c + '_kt', 'run_kernel_stats.csv')} {os.path.join(dst, c + '_kernel_stats.csv')}")
    summary[c] = {k: d[k] for k in ("traffic_over_alg", "fetch_bytes_per_packet", "atomics_per_packet", "sq_wait_any_frac",
                                    "kernel_trace_avg_ms")}

na = bench_line("c5_noatomic.log")
c3 = [bench_line(f"c3_rep{k}.log") for k in (1, 2, 3)]
summary["c5_map_adds_compiled_out_kernel_ms"] = na["roofline"]["avg_kernel_ms"] if na else None
summary["c3_kernel_ms_per_process"] = [x["roofline"]["kernel_ms_steps"] for x in c3 if x]
json.dump(summary, open(os.path.join(dst, "counters_summary.json"), "w"), indent=1)
print(json.dumps(summary, indent=1))
