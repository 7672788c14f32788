#!/bin/bash
# Round 2, GPU call 5: paired deferral of 8-byte map adds (C5), C3 with 4 replicas: parity suite,
# then C5 / C3 / C2 bench lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/r2g5; mkdir -p $OUT
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -25 $OUT/$name.log; exit 1; }
}
K='"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"avg_kernel_ms": [0-9.]*\|"frac": [0-9.]*'
step c5 240 python bench.py --config c5 --steps 6 --warmup 2 --no-cpu-baseline --no-e2e
grep -o "$K" $OUT/c5.log | tr '\n' ' '; echo
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
tail -1 $OUT/pytest_gpu.log
for k in 1 2; do
  step c3_$k 240 python bench.py --config c3 --steps 8 --warmup 2 --no-cpu-baseline --no-e2e
  grep -o "$K" $OUT/c3_$k.log | tr '\n' ' '; echo
done
step c2 240 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-ordered
grep -o "$K" $OUT/c2.log | tr '\n' ' '; echo
echo done
