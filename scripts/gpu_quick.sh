#!/bin/bash
# parity tests then a short multi-config bench sweep (each step time-limited; stop at first failure)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/q
timeout -k 10 900 python -m pytest tests -m gpu -x -q ${PYTEST_ARGS} > gpurun_out/q/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/q/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for cfg in $(echo ${CFGS:-c1:16777216,c2:16777216,c4:1048576} | tr ',' ' '); do
  set -- ${cfg%%:*} ${cfg##*:}
  for eng in ${ENGINES:-jit interp}; do
    timeout -k 10 300 python bench.py --config $1 --packets $2 --steps 5 --warmup 1 --engine $eng --no-cpu-baseline > gpurun_out/q/bench_${1}_${eng}.log 2>&1 || { echo "bench $1 $eng failed"; tail -3 gpurun_out/q/bench_${1}_${eng}.log; exit 1; }
    echo "$1 $eng $(tail -1 gpurun_out/q/bench_${1}_${eng}.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], "Mpkt/s kernel_ms", d["roofline"]["avg_kernel_ms"], "frac", d["roofline"]["frac"])')"
  done
done
