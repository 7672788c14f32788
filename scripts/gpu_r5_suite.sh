#!/bin/bash
# Round 5: the whole -m gpu suite on the in-tree build (no rebuild on the box: XE_SKIP_PRODUCT_BUILD).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5suite}; mkdir -p $OUT
export XE_SKIP_PRODUCT_BUILD=1
# a test that compiles kernels it finds in no cache prints nothing for minutes (pytest -v reports at its
# end): a heartbeat under gpurun_out/ keeps the silence watchdog off it; --timeout bounds each test
( while sleep 50; do date +%T >> $OUT/heartbeat; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 1080 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|^E " $OUT/pytest.log | head -20; exit 1; }
