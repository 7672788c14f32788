#!/bin/bash
# Round 2, GPU call 7: fused batch tail with burst atomics (C2 pipelined vs synchronous, kernel
# trace), then the C3 mode differential: C3 bench processes under one TCC pass and one SQ pass each.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/r2g7; mkdir -p $OUT
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -30 $OUT/$name.log; exit 1; }
}
K='"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"avg_kernel_ms": [0-9.]*\|"frac": [0-9.]*'
step pytest_async 300 python -u -m pytest tests/test_async.py -m gpu -x -v --timeout 200 --timeout-method thread
tail -1 $OUT/pytest_async.log
step c2_pipe 240 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-ordered
grep -o "$K" $OUT/c2_pipe.log | tr '\n' ' '; echo
step c2_sync 240 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-ordered --sync
grep -o "$K" $OUT/c2_sync.log | tr '\n' ' '; echo
step c2_kt 240 rocprofv3 --kernel-trace --stats -d $OUT/c2_kt -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-ordered
grep -o "$K" $OUT/c2_kt.log | tr '\n' ' '; echo
B="--config c3 --steps 6 --warmup 2 --no-cpu-baseline --no-e2e"
for k in 1 2 3 4 5; do
  step c3_tcc$k 240 rocprofv3 --pmc TCC_EA0_ATOMIC_sum TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum -d $OUT/c3_tcc$k -o run --output-format csv -- python3 bench.py $B
  grep -o '"avg_kernel_ms": [0-9.]*' $OUT/c3_tcc$k.log
done
for k in 1 2 3 4 5; do
  step c3_sq$k 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INSTS_VALU -d $OUT/c3_sq$k -o run --output-format csv -- python3 bench.py $B
  grep -o '"avg_kernel_ms": [0-9.]*' $OUT/c3_sq$k.log
done
echo done
