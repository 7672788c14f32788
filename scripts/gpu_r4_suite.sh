#!/bin/bash
# Round 4: the -m gpu suite, smoke(), and the default bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/r4s; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=8 -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $OUT/pytest_gpu.log | head -20; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && tail -1 $OUT/smoke.log &&
timeout -k 10 420 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err && echo bench ok
