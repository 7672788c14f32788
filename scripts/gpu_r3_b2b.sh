#!/bin/bash
# bpf2bpf (dynamic block form, general lane model) at 2 waves per SIMD: the call / tail-call parity
# tests on device, the bench line, and the kernel stats. Usage: gpu_r3_b2b.sh TAG
set -o pipefail
OUT=gpurun_out/$1; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "bpf2bpf or call or tail or frame" > $OUT/pytest_calls.txt 2>&1 || { tail -20 $OUT/pytest_calls.txt; exit 1; }
tail -2 $OUT/pytest_calls.txt
timeout -k 10 300 python bench.py --config bpf2bpf --engine jit --no-cpu-baseline --no-e2e --no-ordered \
  > $OUT/bench_bpf2bpf.json 2> $OUT/bench_bpf2bpf.err || { tail -5 $OUT/bench_bpf2bpf.err; exit 1; }
cat $OUT/bench_bpf2bpf.json
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/b2b_stats -o run --output-format csv -- python3 bench.py --config bpf2bpf \
  --engine jit --steps 10 --no-cpu-baseline --no-e2e --no-ordered > $OUT/b2b_bench_under_rocprof.json 2> $OUT/b2b_stats.err \
  || { tail -5 $OUT/b2b_stats.err; exit 1; }
echo rocprof done
