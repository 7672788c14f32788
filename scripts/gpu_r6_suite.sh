#!/bin/bash
# Round 6: the whole -m gpu suite on the in-tree build and the in-tree ahead-of-time kernel cache
# (python -m gobpfld_amd.aot, built on the CPU machine). No heartbeat: a test that compiled a kernel
# itself is named in the suite's "per-program kernels" summary with the seconds it spent, and
# --durations=15 names the slowest tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r6suite}; mkdir -p $OUT
export XE_SKIP_PRODUCT_BUILD=1
timeout -k 10 1080 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=15 \
  ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/pytest.log 2>&1; rc=$?
tail -40 $OUT/pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|^E " $OUT/pytest.log | head -20; exit 1; }
