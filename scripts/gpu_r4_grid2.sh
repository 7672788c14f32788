#!/bin/bash
# Grid A/B after key shadows (C5 48 VGPRs, memory-latency bound): 4 vs 5 resident blocks per CU
# (XE_MAX_BLOCKS through the tuning build) for C5 and C3, one process per variant.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/r4grid2; mkdir -p $OUT
TLIB=$PWD/gobpfld_amd/libxdpemu_tuning.so
run() {  # cfg blocks
  XE_LIB=$TLIB XE_MAX_BLOCKS=$2 timeout -k 10 200 python bench.py --config $1 --no-c5 --no-ordered --no-e2e --no-cpu-baseline > $OUT/$1_mb$2.json 2> $OUT/$1_mb$2.err || { tail -3 $OUT/$1_mb$2.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], sys.argv[3], d['config'].get('grid'), r['avg_kernel_ms'], r['frac'], d.get('verified'))" $OUT/$1_mb$2.json $1 $2
}
for mb in 1024 1280 1024 1280; do run c5 $mb || exit 1; done
for mb in 1024 1280; do run c3 $mb || exit 1; done

# keyed C3-LRU: kernel breakdown (product build) and the keyed attempt trace (tuning build)
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_c3lru -o run --output-format csv -- python3 scripts/prof_c3lru.py > $OUT/prof_c3lru.log 2>&1 || { echo "prof c3lru failed"; tail -3 $OUT/prof_c3lru.log; exit 1; }
tail -1 $OUT/prof_c3lru.log
XE_LIB=$TLIB XE_KEYED_TRACE=1 timeout -k 10 300 python3 scripts/prof_c3lru.py > $OUT/trace_c3lru.log 2>&1 || { echo "trace c3lru failed"; tail -3 $OUT/trace_c3lru.log; exit 1; }
grep -c keyed $OUT/trace_c3lru.log; grep keyed $OUT/trace_c3lru.log | sort | uniq -c | head
echo all done
