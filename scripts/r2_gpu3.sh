#!/bin/bash
# Round 2, GPU call 3: parity suite (pipelined batches, 64-B probe groups), C2 pipelined vs synchronous
# steps, C5 with the 64-B probe group and its adds compiled out, the C3 placement experiment.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/r2g3; mkdir -p $OUT
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -25 $OUT/$name.log; exit 1; }
}
step pytest_async 300 python -u -m pytest tests/test_async.py -m gpu -x -v --timeout 200 --timeout-method thread
tail -1 $OUT/pytest_async.log
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
tail -1 $OUT/pytest_gpu.log
step c2_pipe 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-ordered
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"avg_kernel_ms": [0-9.]*' $OUT/c2_pipe.log | tr '\n' ' '; echo
step c2_sync 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-ordered --sync
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"avg_kernel_ms": [0-9.]*' $OUT/c2_sync.log | tr '\n' ' '; echo
step c5 240 python bench.py --config c5 --steps 6 --warmup 2 --no-cpu-baseline --no-e2e
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"avg_kernel_ms": [0-9.]*' $OUT/c5.log | tr '\n' ' '; echo
XE_LIB=gobpfld_amd/libxdpemu_tuning.so XE_JIT_DEFINES=-DXE_DEBUG_NO_ATOMIC=1 step c5_noatomic 240 python bench.py --config c5 --steps 6 --warmup 2 --no-cpu-baseline --no-e2e
grep -o '"avg_kernel_ms": [0-9.]*' $OUT/c5_noatomic.log
step c3_placement 400 python -u scripts/c3_placement.py
grep trial $OUT/c3_placement.log
echo done
