#!/bin/bash
# Round 2, GPU call 9: one-block epilogue launch per pipelined batch (records to pinned host memory,
# replay decision, small-map fold + next snapshot), shard epochs: async tests, C2 pipelined /
# synchronous with a kernel trace, C5, C3, then the whole parity suite.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/r2g9; mkdir -p $OUT
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
step c5 240 python bench.py --config c5 --steps 6 --warmup 2 --no-cpu-baseline --no-e2e
grep -o "$K" $OUT/c5.log | tr '\n' ' '; echo
step c3 240 python bench.py --config c3 --steps 8 --warmup 2 --no-cpu-baseline --no-e2e
grep -o "$K" $OUT/c3.log | tr '\n' ' '; echo
step c4 240 python bench.py --config c4 --steps 8 --warmup 2 --no-cpu-baseline --no-e2e
grep -o "$K" $OUT/c4.log | tr '\n' ' '; echo
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
tail -1 $OUT/pytest_gpu.log
echo done
