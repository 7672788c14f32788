#!/bin/bash
# Round 6: occupancy A/B of the issue/latency-bound configs (C4 97 VGPRs = 4 waves/SIMD, C5 / C3 90 = 5):
# the per-program kernel compiled for more waves per SIMD (XE_MIN_WAVES_PER_EU), tuning build, one bench
# process per variant (scripts/gpu_ab.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
bash scripts/gpu_ab.sh r6occ "c4" "" "-DXE_MIN_WAVES_PER_EU=5" "-DXE_MIN_WAVES_PER_EU=6" || exit 1
bash scripts/gpu_ab.sh r6occ "c5 c3" "" "-DXE_MIN_WAVES_PER_EU=6" || exit 1
