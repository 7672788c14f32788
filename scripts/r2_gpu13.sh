#!/bin/bash
# Round 2, GPU call 13: header reads at constant LDS offsets when the chunk's packets are 16-B aligned
# (wave-uniform): C2 bench + SQ pass, C3/C4/C5 bench lines, the parity suite.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/r2g13; mkdir -p $OUT
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  timeout -k 10 -s KILL $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -30 $OUT/$name.log; exit 1; }
}
K='"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"avg_kernel_ms": [0-9.]*\|"frac": [0-9.]*'
step c2 240 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-ordered
grep -o "$K" $OUT/c2.log | tr '\n' ' '; echo
step c2_sq 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INSTS_VALU -d $OUT/c2_sq -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-e2e --no-ordered --sync
for c in c5 c4 c3; do
  step $c 240 python bench.py --config $c --steps 8 --warmup 2 --no-cpu-baseline --no-e2e
  grep -o "$K" $OUT/$c.log | tr '\n' ' '; echo
done
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
tail -1 $OUT/pytest_gpu.log
echo done
