#!/bin/bash
# Round 5: the whole -m gpu suite on the in-tree build (no rebuild on the box: XE_SKIP_PRODUCT_BUILD).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5suite}; mkdir -p $OUT
export XE_SKIP_PRODUCT_BUILD=1
timeout -k 10 1080 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|^E " $OUT/pytest.log | head -20; exit 1; }
