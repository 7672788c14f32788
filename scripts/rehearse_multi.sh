#!/bin/bash
# Rehearsal of bench.py's N > 1 path (one process per GPU, shard epoch: footprint all-gather, check,
# per-map delta all-reduce, then the self-check against header truth) with 2 ranks sharing the one GPU of
# a gpurun box over gloo, started the way `bench.py --gpus 2` starts them. Checks that the step path runs,
# reports its exchanges and verifies; the throughput of such a run is meaningless.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/rehearse; mkdir -p $OUT
XE_BENCH_REHEARSE=1 timeout -k 10 -s KILL 300 python bench.py --gpus 2 --steps 4 --warmup 1 --packets 1048576 \
  --c5-packets 1048576 --c5-steps 2 --no-cpu-baseline --no-e2e --no-ordered > $OUT/c2_2ranks.log 2>&1
rc=$?; echo "c2_2ranks rc=$rc"; tail -3 $OUT/c2_2ranks.log | cut -c1-900; [ $rc -eq 0 ] || exit 1
XE_BENCH_REHEARSE=1 timeout -k 10 -s KILL 300 python bench.py --gpus 2 --config c3 --steps 3 --warmup 1 --packets 1048576 \
  --no-cpu-baseline --no-e2e > $OUT/c3_2ranks.log 2>&1
rc=$?; echo "c3_2ranks rc=$rc"; tail -3 $OUT/c3_2ranks.log | cut -c1-600; [ $rc -eq 0 ] || exit 1
echo done
