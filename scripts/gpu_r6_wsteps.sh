#!/bin/bash
# Round 6: wave step counts in the verdict-only variant (xe_jit.cpp emit_body_blocks): the step-total
# parity tests, C4 full size, then the C4 line on the product build and the XE_WSTEPS=0 A/B (tuning build)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r6ws}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_wave_steps.py \
  tests/test_gpu_fullsize.py tests/test_gpu_parity.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
bash scripts/gpu_ab.sh ${TAG:-r6ws} "c4" "" "-DXE_WSTEPS=0" "" "-DXE_MIN_WAVES_PER_EU=5" || exit 1
