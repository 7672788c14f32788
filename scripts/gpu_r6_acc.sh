#!/bin/bash
# Round 6: what C5's accumulator-table probes cost (XE_ACC_BYPASS: 8-byte adds straight to the paired
# block, exact) against the default, C5 and C2 (whose hot counters need the table), tuning build
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
bash scripts/gpu_ab.sh ${TAG:-r6acc} "c5 c2" "" "-DXE_ACC_BYPASS" "" "-DXE_ACC_BYPASS" || exit 1
