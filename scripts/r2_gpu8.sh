#!/bin/bash
# Round 2, GPU call 8: batch tail without the per-block release (async tests, C2 pipelined /
# synchronous), and C2 at 3 waves per SIMD (is the kernel latency-bound?).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/r2g8; mkdir -p $OUT
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
XE_LIB=gobpfld_amd/libxdpemu_tuning.so XE_JIT_DEFINES=-DXE_MIN_WAVES_PER_EU=3 step c2_w3 240 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-ordered --sync
grep -o "$K" $OUT/c2_w3.log | tr '\n' ' '; echo
step c5 240 python bench.py --config c5 --steps 6 --warmup 2 --no-cpu-baseline --no-e2e
grep -o "$K" $OUT/c5.log | tr '\n' ' '; echo
echo done
