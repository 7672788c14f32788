#!/bin/bash
# C3 / C4 twice each in fresh processes (run-to-run modes).
set -e
OUT=gpurun_out/r2c34
mkdir -p $OUT
for k in 1 2; do for c in c3 c4; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-e2e --steps 10 > $OUT/bench_${c}_$k.json 2> $OUT/bench_${c}_$k.err || { tail -5 $OUT/bench_${c}_$k.err; exit 1; }
done; done
echo ok
