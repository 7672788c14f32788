#!/bin/bash
# Round 2, GPU call 1: GPU parity suite (general lane model, calls/tail calls/ordered maps, the two-shard
# device exchange), smoke, the C2 and C1 bench lines, and the C3 replica-skew A/B (per-process placement
# hypothesis for C3's bimodality).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/r2g1; mkdir -p $OUT
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -25 $OUT/$name.log; exit 1; }
}
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
tail -3 $OUT/pytest_gpu.log
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_c2 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e
grep '"metric"' $OUT/bench_c2.log | cut -c1-600
step bench_c1 300 python bench.py --config c1 --steps 10 --warmup 2 --no-e2e
grep '"metric"' $OUT/bench_c1.log | cut -c1-600
for skew in 0 1280 0 1280 0 1280; do
  XE_LIB=gobpfld_amd/libxdpemu_tuning.so XE_REP_SKEW=$skew step c3_skew$skew 240 python bench.py --config c3 --steps 6 --warmup 2 --no-cpu-baseline --no-e2e
  grep -o '"avg_kernel_ms": [0-9.]*' $OUT/c3_skew$skew.log | sed "s/^/skew $skew /"
done
echo done
