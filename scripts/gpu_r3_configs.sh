#!/bin/bash
# Round-3 bench lines for C1-C5 (one process each, own time limit) after the suite check.
set -o pipefail
OUT=gpurun_out/${1:-r3cfg}
mkdir -p $OUT
for cfg in "c2" "c3" "c4" "c5 --packets 33554432" "c1" "bpf2bpf --engine jit"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --config $cfg --no-cpu-baseline --no-e2e --no-ordered > $OUT/bench_$1.json 2> $OUT/bench_$1.err || { tail -5 $OUT/bench_$1.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], d['value'], 'Mpkt/s kernel', r['avg_kernel_ms'], 'frac', r['frac'])" $OUT/bench_$1.json $1
done
