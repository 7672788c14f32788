#!/bin/bash
# Round-3 evidence: rocprofv3 kernel stats of the default bench command, the keyed C3-learn timeline at
# 16M packets, and the window A/B per config (tuning build). Each GPU step under its own limit.
set -o pipefail
T=${1:-r3prof}
OUT=gpurun_out/$T; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/c2_stats -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-e2e --no-ordered > $OUT/c2_bench_under_rocprof.json 2> $OUT/c2_stats.err || { tail -5 $OUT/c2_stats.err; exit 1; }
echo "c2 rocprof done"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/keyed16 -o run --output-format csv -- python3 scripts/keyed_profile.py 16777216 3 > $OUT/keyed16.log 2>&1 || { tail -5 $OUT/keyed16.log; exit 1; }
tail -3 $OUT/keyed16.log
echo "keyed done"
bash scripts/gpu_ab.sh ${T}_ab2 "c2" "" "-DXE_HDR_LO=0 -DXE_HDR_HI=28" "-DXE_HDR_LO=0 -DXE_HDR_HI=64" || exit 1
bash scripts/gpu_ab.sh ${T}_ab3 "c3 c4 c5:33554432" "" "-DXE_HDR_LO=0 -DXE_HDR_HI=42" "-DXE_HDR_LO=0 -DXE_HDR_HI=64" "-DXE_MIN_WAVES_PER_EU=5" || exit 1
