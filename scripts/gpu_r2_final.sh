#!/bin/bash
# Round-2 final evidence on one MI355X: GPU parity suite, the default bench line (as the driver runs
# it), and the kernel-trace statistics of the same bench command. Each step under its own time limit.
set -e
OUT=gpurun_out/r2final
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -20 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-e2e > $OUT/bench_kt.json 2> $OUT/bench_kt.err || { tail -5 $OUT/bench_kt.err; exit 1; }
echo ok
