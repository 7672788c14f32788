#!/bin/bash
# Round 5: quick measurement pass after a change — the keyed streams (per-dispatch trace), the one-lane
# replay rates, and the C2 / C4 / C5 kernel times from bench.py single-config lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
T=${TAG:-r5q}
CONFIGS="${KCONF:-c3lru c3learn}" TAG=${T}_kp scripts/gpu_r5_keyedprof.sh || exit 1
NO_SQ=1 CONFIGS="${SCONF:-c2rmw c3learn c3lru c3lrufull}" TAG=${T}_seq scripts/gpu_r5_seq.sh || exit 1
OUT=gpurun_out/$T; mkdir -p $OUT
B="--no-cpu-baseline --no-e2e --no-ordered --no-c5 --no-c4"
for c in ${BCONF:-c4 c2 c5}; do
  timeout -k 10 300 python bench.py --config $c $B > $OUT/bench_$c.json 2> $OUT/bench_$c.err || { echo "bench $c failed"; tail -3 $OUT/bench_$c.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['roofline']['avg_kernel_ms'], d['roofline']['frac'], d['verified'])" $OUT/bench_$c.json $c
done
echo quick done
