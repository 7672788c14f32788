#!/bin/bash
# Round 2, GPU call 3: C3 placement experiment (VM vs UMEM re-allocation in one process), C5 with the
# 64-B probe group (default) and its map adds compiled out (cost split).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/r2g3; mkdir -p $OUT
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -25 $OUT/$name.log; exit 1; }
}
step c3_placement 400 python -u scripts/c3_placement.py
cat $OUT/c3_placement.log | grep trial
step c5 240 python bench.py --config c5 --steps 6 --warmup 2 --no-cpu-baseline --no-e2e
grep -o '"avg_kernel_ms": [0-9.]*' $OUT/c5.log
XE_LIB=gobpfld_amd/libxdpemu_tuning.so XE_JIT_DEFINES=-DXE_DEBUG_NO_ATOMIC=1 step c5_noatomic 240 python bench.py --config c5 --steps 6 --warmup 2 --no-cpu-baseline --no-e2e
grep -o '"avg_kernel_ms": [0-9.]*' $OUT/c5_noatomic.log
echo done
