#!/bin/bash
# Round 2, GPU call 14: staged sequential replay (the wave stages 64 packets, lane 0 runs them):
# parity suite, then the C2 bench with its ordered-path lines (C2-RMW lifted / one lane).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/r2g14; mkdir -p $OUT
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  timeout -k 10 -s KILL $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -30 $OUT/$name.log; exit 1; }
}
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
tail -1 $OUT/pytest_gpu.log
step c2_full 400 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"sequential_one_lane": {[^}]*}' $OUT/c2_full.log | tr '\n' ' '; echo
echo done
