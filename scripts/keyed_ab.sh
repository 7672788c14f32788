#!/bin/bash
# A/B of the keyed variant's occupancy bound (tuning library, XE_JIT_DEFINES): per-kernel times of a
# C3-learn keyed run, 4 waves / SIMD (spills) vs 3 waves / SIMD (no spills). GPU box only.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export XE_LIB=$GRAFT_REPO_ROOT/gobpfld_amd/libxdpemu_tuning.so
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/kab4 -o run -- python3 scripts/keyed_profile.py 4194304 4 > gpurun_out/kab4.log 2>&1
XE_JIT_DEFINES="-DXE_MIN_WAVES_PER_EU=3" timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/kab3 -o run -- python3 scripts/keyed_profile.py 4194304 4 > gpurun_out/kab3.log 2>&1
grep mpkts gpurun_out/kab4.log gpurun_out/kab3.log
