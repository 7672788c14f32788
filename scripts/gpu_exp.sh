#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/misc
timeout -k 10 120 rocprofv3 -L > gpurun_out/misc/counters.txt 2>&1 || true
export XE_JIT_DEFINES=-DXE_ACC=128
TAG=sq_c3 BENCH_ARGS="--config c3 --steps 2 --warmup 1 --no-cpu-baseline" EXTRA_GROUPS="FETCH_SIZE WRITE_SIZE" bash scripts/prof_sq.sh || exit 1
python3 scripts/pmc_summary.py gpurun_out/sq_c3/pmc*/run_counter_collection.csv
export XE_JIT_DEFINES="-DXE_ACC=128 -DXE_DEBUG_NO_ATOMIC=1"
TAG=sq_c3na BENCH_ARGS="--config c3 --steps 2 --warmup 1 --no-cpu-baseline" bash scripts/prof_sq.sh || exit 1
python3 scripts/pmc_summary.py gpurun_out/sq_c3na/pmc*/run_counter_collection.csv
