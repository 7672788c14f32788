#!/bin/bash
# Iteration check: GPU parity tests, then one bench line per config (each step time-limited).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/${TAG:-iter}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_ARGS} > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for c in ${CFGS:-c2 c3 c4 c5}; do
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_$c.log 2>&1 || { echo "bench $c failed"; tail -3 $OUT/bench_$c.log; exit 1; }
  echo "$c $(tail -1 $OUT/bench_$c.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], "Mpkt/s kernel_ms", r["avg_kernel_ms"], "frac", r["frac"], "grid", d["config"].get("grid"))')"
done
