#!/bin/bash
# A/B of environment variants over configs: VARIANTS="name=ENV=VAL ENV2=VAL;name2=..." (empty env ok)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/ab; mkdir -p $OUT
if [ -n "$WITH_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
IFS=';' read -ra VS <<< "${VARIANTS:-base=}"
for v in "${VS[@]}"; do
  vn=${v%%=*}; envs=${v#*=}
  for c in ${CFGS:-c2 c3 c4 c5}; do
    env $envs timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline > $OUT/${vn}_$c.log 2>&1 || { echo "bench $vn $c failed"; tail -3 $OUT/${vn}_$c.log; exit 1; }
    echo "$vn $c $(tail -1 $OUT/${vn}_$c.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], "Mpkt/s kernel_ms", r["avg_kernel_ms"], "frac", r["frac"], "grid", d["config"].get("grid"))')"
  done
done
