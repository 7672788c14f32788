#!/bin/bash
# C3 run-to-run modes: ten fresh processes (new map allocations each), one bench line each.
set -o pipefail
OUT=gpurun_out/${1:-c3modes}; mkdir -p $OUT
for i in 1 2 3 4 5 6 7 8 9 10; do
  timeout -k 10 240 python bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-ordered > $OUT/c3_$i.json 2> $OUT/c3_$i.err || { tail -5 $OUT/c3_$i.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('run', sys.argv[2], d['value'], 'Mpkt/s kernel', d['roofline']['avg_kernel_ms'])" $OUT/c3_$i.json $i
done
