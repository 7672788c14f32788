#!/bin/bash
# Round 4, keyed C3-LRU: the ordered-map device tests, then the C3-LRU keyed batch under rocprofv3
# (kernels + HIP API calls, to see the host gaps between the passes).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/r4lru; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_ordered_par.py tests/test_lru_golden.py tests/test_keyed.py -m gpu --maxfail=5 -v --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|^E " $OUT/pytest.log | head -20; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-trace --hip-trace --stats -d $OUT/prof_c3lru -o run --output-format csv -- python3 scripts/prof_c3lru.py > $OUT/prof_c3lru.log 2>&1 || { echo "prof c3lru failed"; tail -3 $OUT/prof_c3lru.log; exit 1; }
grep keyed $OUT/prof_c3lru.log | tail -1
XE_LIB=$PWD/gobpfld_amd/libxdpemu_tuning.so XE_HOST_TIMING=1 timeout -k 10 300 python3 scripts/prof_c3lru.py > $OUT/host.log 2>&1 || { tail -5 $OUT/host.log; exit 1; }
grep -v "n=0)" $OUT/host.log | tail -12
echo all done
