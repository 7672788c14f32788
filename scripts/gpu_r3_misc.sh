#!/bin/bash
# occupancy A/B (tuning build), C3 run-to-run modes, and the 2-rank rehearsal of the N > 1 bench path.
set -o pipefail
T=${1:-r3misc}
bash scripts/gpu_ab.sh ${T}_occ "c2" "" "-DXE_MIN_WAVES_PER_EU=6" "-DXE_MIN_WAVES_PER_EU=7" "-DXE_MIN_WAVES_PER_EU=8" || exit 1
bash scripts/c3_modes.sh ${T}_c3modes || exit 1
bash scripts/rehearse_multi.sh || exit 1
