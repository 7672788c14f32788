#!/bin/bash
# instruction-mix counters for C1 (fixed per-chunk overhead) and C2
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
for c in c1 c2 c4; do
  TAG=sq_$c BENCH_ARGS="--config $c --packets 16777216 --steps 3 --warmup 1 --no-cpu-baseline" bash scripts/prof_sq.sh || exit 1
  python3 scripts/pmc_summary.py gpurun_out/sq_$c/pmc*/run_counter_collection.csv
done
