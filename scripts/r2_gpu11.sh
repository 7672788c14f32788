#!/bin/bash
# Round 2, GPU call 11: deferred verdict / paired-add commit (one chunk later, behind the next
# prefetch): parity suite, then C2/C5/C3/C4 with the commit deferred and (tuning build) not.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/r2g11; mkdir -p $OUT
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -30 $OUT/$name.log; exit 1; }
}
K='"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"avg_kernel_ms": [0-9.]*\|"frac": [0-9.]*'
step c2 240 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-ordered
grep -o "$K" $OUT/c2.log | tr '\n' ' '; echo
XE_LIB=gobpfld_amd/libxdpemu_tuning.so XE_JIT_DEFINES=-DXE_DEFER_COMMIT=0 step c2_nodefer 240 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-ordered
grep -o "$K" $OUT/c2_nodefer.log | tr '\n' ' '; echo
step c5 240 python bench.py --config c5 --steps 6 --warmup 2 --no-cpu-baseline --no-e2e
grep -o "$K" $OUT/c5.log | tr '\n' ' '; echo
XE_LIB=gobpfld_amd/libxdpemu_tuning.so XE_JIT_DEFINES=-DXE_DEFER_COMMIT=0 step c5_nodefer 240 python bench.py --config c5 --steps 6 --warmup 2 --no-cpu-baseline --no-e2e
grep -o "$K" $OUT/c5_nodefer.log | tr '\n' ' '; echo
step c4 240 python bench.py --config c4 --steps 8 --warmup 2 --no-cpu-baseline --no-e2e
grep -o "$K" $OUT/c4.log | tr '\n' ' '; echo
step c3 240 python bench.py --config c3 --steps 8 --warmup 2 --no-cpu-baseline --no-e2e
grep -o "$K" $OUT/c3.log | tr '\n' ' '; echo
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -rs --timeout 300 --timeout-method thread
tail -3 $OUT/pytest_gpu.log
echo done
