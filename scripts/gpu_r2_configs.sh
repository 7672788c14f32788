#!/bin/bash
# C3 / C4 / C5 bench lines on the final round-2 tree (no CPU baseline / e2e side lines).
set -e
OUT=gpurun_out/r2configs
mkdir -p $OUT
for c in c3 c4 c5; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-e2e > $OUT/bench_$c.json 2> $OUT/bench_$c.err || { tail -5 $OUT/bench_$c.err; exit 1; }
done
echo ok
