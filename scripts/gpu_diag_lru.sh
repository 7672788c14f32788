#!/bin/bash
# Diagnose the LRU keyed-path failure on the device: which earlier tests make it appear.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/diag; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "kat" -v --maxfail=3 --timeout 120 --timeout-method thread > $OUT/kats.log 2>&1
echo "kats rc=$?"; grep -E "FAIL|rror" $OUT/kats.log | head -20
timeout -k 10 500 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_multi.py tests/test_gpu_parity.py -k "fullsize or multi or lru_evicts" -v --maxfail=3 --timeout 200 --timeout-method thread > $OUT/seq.log 2>&1
echo "seq rc=$?"; grep -E "PASS|FAIL|rror" $OUT/seq.log | head -40
