#!/bin/bash
# GPU validation + bench: each GPU step under its own time limit, stop at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
for eng in ${ENGINES:-jit interp}; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --engine $eng --no-cpu-baseline > gpurun_out/bench_$eng.log 2>&1
  rc=$?; echo "bench $eng rc=$rc"; tail -1 gpurun_out/bench_$eng.log | cut -c1-600
  [ $rc -eq 0 ] || exit $rc
done
