#!/bin/bash
# Round 4, first box: C2 speed of light (tools/sol_c2), the default bench (verified + c5 side line),
# C2 --sync vs pipelined and C2-RMW pipelined (the C2 vs C2-RMW kernel-time question), the 2-rank rehearsal.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/r4a; mkdir -p $OUT
timeout -k 10 120 tools/sol_c2 > $OUT/sol_c2.jsonl 2>&1 && echo sol ok &&
timeout -k 10 420 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err && echo bench ok &&
timeout -k 10 200 python bench.py --sync --no-c5 --no-ordered --no-e2e --no-cpu-baseline > $OUT/bench_c2_sync.json 2>&1 && echo sync ok &&
timeout -k 10 200 python bench.py --config c2rmw --no-ordered --no-e2e --no-cpu-baseline > $OUT/bench_c2rmw.json 2>&1 && echo rmw ok &&
timeout -k 10 200 python bench.py --config c2rmw --sync --no-ordered --no-e2e --no-cpu-baseline > $OUT/bench_c2rmw_sync.json 2>&1 && echo rmwsync ok &&
bash scripts/rehearse_multi.sh
