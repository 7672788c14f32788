#!/bin/bash
# Round 4: the two-rank exchange tests, the rehearsal, and a C2 grid A/B (4 vs 6 blocks per CU).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/r4b; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_multi.py > $OUT/multi.log 2>&1; rc=$?; tail -5 $OUT/multi.log; [ $rc -eq 0 ] || exit 1
bash scripts/rehearse_multi.sh || exit 1
for mb in 1024 1280 1536; do
  XE_MAX_BLOCKS=$mb XE_LIB=$PWD/gobpfld_amd/libxdpemu_tuning.so timeout -k 10 120 python bench.py --no-c5 --no-ordered --no-e2e --no-cpu-baseline > $OUT/c2_mb$mb.json 2>&1 || exit 1
done
grep -ho '"avg_kernel_ms": [0-9.]*' $OUT/c2_mb*.json
