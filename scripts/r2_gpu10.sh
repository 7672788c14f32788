#!/bin/bash
# Round 2, GPU call 10: FETCH_SIZE accounting of the sparse read shapes (tools/calib_fetch2), then the
# final tree's PMC traffic passes (FETCH_SIZE, WRITE_SIZE, separate runs) and kernel stats for the
# C2 bench line, C5, C4 and C3.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/r2g10; mkdir -p $OUT
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  timeout -k 10 -s KILL $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -15 $OUT/$name.log; exit 1; }
}
step calib2_fetch 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/calib2_fetch -o run --output-format csv -- ./tools/calib_fetch2
step calib2_rdreq 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum -d $OUT/calib2_rdreq -o run --output-format csv -- ./tools/calib_fetch2
cat $OUT/calib2_fetch.log | tail -1
for c in c2 c5 c4 c3; do
  B="--config $c --steps 5 --warmup 1 --no-cpu-baseline --no-e2e --no-ordered"
  step ${c}_kt 240 rocprofv3 --kernel-trace --stats -d $OUT/${c}_kt -o run --output-format csv -- python3 bench.py $B
  tail -1 $OUT/${c}_kt.log > $OUT/bench_${c}_under_rocprof.json
  step ${c}_fetch 240 rocprofv3 --pmc FETCH_SIZE -d $OUT/${c}_fetch -o run --output-format csv -- python3 bench.py $B
  step ${c}_write 240 rocprofv3 --pmc WRITE_SIZE -d $OUT/${c}_write -o run --output-format csv -- python3 bench.py $B
  step ${c}_rdreq 240 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_ATOMIC_sum -d $OUT/${c}_rdreq -o run --output-format csv -- python3 bench.py $B
done
echo done
