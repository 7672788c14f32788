#!/bin/bash
# Final round-3 check: suite + smoke + default bench, the C1-C5 and bpf2bpf lines, and the rocprofv3
# kernel stats of the default bench command.
set -o pipefail
T=${1:-r3final}
bash scripts/gpu_r3_suite.sh $T && bash scripts/gpu_r3_configs.sh $T || exit 1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/c2_stats -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-e2e --no-ordered > gpurun_out/$T/c2_bench_under_rocprof.json 2> gpurun_out/$T/c2_stats.err || { tail -5 gpurun_out/$T/c2_stats.err; exit 1; }
echo "rocprof done"
