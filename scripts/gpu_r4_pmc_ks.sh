#!/bin/bash
# PMC traffic of C5 and C3 after key shadows (one counter group per run), for scripts/traffic.py
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/r4pmcks; mkdir -p $OUT
B="--no-cpu-baseline --no-e2e --no-ordered --no-c5 --no-verify"
for cfg in "c5 33554432" "c3 16777216"; do
  set -- $cfg
  for grp in "FETCH_SIZE:fetch" "WRITE_SIZE:write" "TCC_EA0_RDREQ_sum TCC_EA0_ATOMIC_sum:rdreq"; do
    ctrs=${grp%%:*}; tag=${grp##*:}
    timeout -s KILL 120 rocprofv3 --pmc $ctrs -d $OUT/${1}_$tag -o run --output-format csv -- python3 bench.py --config $1 --packets $2 --steps 5 --warmup 1 $B > $OUT/${1}_$tag.log 2>&1 || { echo "pmc $1 $tag failed"; tail -3 $OUT/${1}_$tag.log; exit 1; }
  done
  echo "$1 pmc done"
done
