#!/bin/bash
# Round 4, key shadows (xe_jit.cpp key_shadows): the device parity tests that run per-program kernels
# with HASH lookups, then the C5 / C3 lines, C5's kernel stats and its SQ counters.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/r4ks; mkdir -p $OUT
B="--no-cpu-baseline --no-e2e --no-ordered"
timeout -k 10 600 python -u -m pytest tests/test_key_shadow.py tests/test_gpu_parity.py tests/test_keyed.py -m gpu --maxfail=5 -v --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|^E " $OUT/pytest.log | head -20; exit 1; }
for c in c5 c3; do
  timeout -k 10 240 python bench.py --config $c $B > $OUT/bench_$c.json 2> $OUT/bench_$c.err || { echo "bench $c failed"; tail -5 $OUT/bench_$c.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], d['value'], r.get('avg_kernel_ms'), r.get('frac'), d.get('verified'))" $OUT/bench_$c.json $c
done
timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d $OUT/prof_c5 -o run --output-format csv -- python3 bench.py --config c5 --steps 10 --warmup 2 $B > $OUT/prof_c5.log 2>&1 || { echo "prof c5 failed"; tail -3 $OUT/prof_c5.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY -d $OUT/c5_sq -o run --output-format csv -- python3 bench.py --config c5 --steps 3 --warmup 1 $B --no-verify > $OUT/c5_sq.log 2>&1 || { echo "sq c5 failed"; tail -3 $OUT/c5_sq.log; exit 1; }
echo "all done"
