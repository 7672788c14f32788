#!/bin/bash
# The bpf2bpf line (per-program kernel, dynamic block form) and the rocprofv3 kernel stats of the
# default bench command.
set -o pipefail
T=${1:-r3final}
mkdir -p gpurun_out/$T
timeout -k 10 300 python bench.py --config bpf2bpf --engine jit --no-cpu-baseline --no-e2e --no-ordered > gpurun_out/$T/bench_bpf2bpf.json 2> gpurun_out/$T/bench_bpf2bpf.err || { tail -5 gpurun_out/$T/bench_bpf2bpf.err; exit 1; }
tail -1 gpurun_out/$T/bench_bpf2bpf.json | cut -c1-400
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/c2_stats -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-e2e --no-ordered > gpurun_out/$T/c2_bench_under_rocprof.json 2> gpurun_out/$T/c2_stats.err || { tail -5 gpurun_out/$T/c2_stats.err; exit 1; }
echo "rocprof done"
