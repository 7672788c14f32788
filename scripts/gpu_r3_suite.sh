#!/bin/bash
# Round-3 GPU check of the tree: the -m gpu suite (with per-test durations), smoke() and the default
# bench line, each under its own time limit; the first failure ends the call.
set -o pipefail
OUT=gpurun_out/${1:-r3suite}
mkdir -p $OUT
t0=$(date +%s)
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=60 > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
echo "suite wall $(( $(date +%s) - t0 )) s"
tail -3 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
