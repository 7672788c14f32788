#!/bin/bash
# Round 6: probe prefetch (xe_interp.h probe_prefetch, xe_jit.cpp pf_plan) A/B on C5 and C3: the
# default kernel (prefetch on) against -DXE_PF=0, twice each, tuning build, one bench process per run
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
bash scripts/gpu_ab.sh ${TAG:-r6pf} "c5 c3" "" "-DXE_PF=0" "" "-DXE_PF=0" || exit 1
