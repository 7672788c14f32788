#!/bin/bash
# A/B of JIT compile-time variants (XE_JIT_DEFINES) over configs: VARIANTS="name=defs;name=defs"
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/ab
IFS=';' read -ra VS <<< "${VARIANTS}"
for v in "${VS[@]}"; do
  vn=${v%%=*}; defs=${v#*=}
  for cfg in $(echo ${CFGS:-c2:16777216,c3:16777216,c5:16777216} | tr ',' ' '); do
    set -- ${cfg%%:*} ${cfg##*:}
    XE_JIT_DEFINES="$defs" timeout -k 10 300 python bench.py --config $1 --packets $2 --steps 5 --warmup 1 --engine jit --no-cpu-baseline > gpurun_out/ab/${vn}_$1.log 2>&1 || { echo "bench $vn $1 failed"; tail -3 gpurun_out/ab/${vn}_$1.log; exit 1; }
    echo "$vn $1 $(tail -1 gpurun_out/ab/${vn}_$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], "Mpkt/s kernel_ms", d["roofline"]["avg_kernel_ms"])')"
  done
done
