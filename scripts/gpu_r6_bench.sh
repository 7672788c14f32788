#!/bin/bash
# Round 6: the default bench line (what the driver runs), then rocprofv3 kernel stats of each config's
# kernel alone (the per-program kernels are all named xe_jit_kernel: one run per config).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r6bench}; mkdir -p $OUT
timeout -k 10 600 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail -20 $OUT/bench_default.err; exit 1; }
cut -c1-400 $OUT/bench_default.json
ONLY="--no-cpu-baseline --no-e2e --no-ordered --no-c3 --no-c4 --no-c5"
for cfg in ${CONFIGS:-"c2:16777216" "c3:16777216" "c4:16777216" "c5:33554432"}; do
  c=${cfg%%:*}; n=${cfg##*:}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$c -o run --output-format csv -- python3 bench.py --config $c --packets $n --steps 20 --warmup 3 $ONLY > $OUT/bench_$c.json 2> $OUT/bench_$c.err || { tail -5 $OUT/bench_$c.err; exit 1; }
  echo "$c profiled"
done
