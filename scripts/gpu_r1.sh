#!/bin/bash
# Round-1 evidence run: GPU parity tests, default bench line (with CPU baseline), rocprof kernel trace
# of the same command, FETCH_SIZE / WRITE_SIZE PMC passes, then the other configs. Each GPU step has
# its own time limit; the script stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r1}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS} > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1 || { echo bench failed; tail -5 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python3 bench.py --no-cpu-baseline > $OUT/bench_kt.log 2>&1 || { echo kt failed; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/pmc_fetch.log 2>&1 || { echo fetch failed; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/pmc_write.log 2>&1 || { echo write failed; exit 1; }
for c in c1 c3 c4 c5; do
  timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline > $OUT/bench_$c.log 2>&1 || { echo "bench $c failed"; tail -3 $OUT/bench_$c.log; exit 1; }
  tail -1 $OUT/bench_$c.log | cut -c1-300
done
echo done
