#!/bin/bash
# Round-2 counter evidence for C3/C4/C5 (VERDICT r1 "next" item 3) + FETCH_SIZE calibration.
# Per config: kernel-trace stats, FETCH_SIZE pass, WRITE_SIZE pass, TCC atomic/hit/miss pass, SQ
# wait pass; then C5 with map adds compiled out (cost split) and three C3 repeats (bimodality).
# Every GPU step has its own limit; the script stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/r2c; mkdir -p $OUT
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  timeout -k 10 -s KILL $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/$name.log; exit 1; }
}
timeout -k 5 60 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
step calib_plain 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/calib -o run --output-format csv -- ./tools/calib_fetch
for c in c3 c4 c5; do
  B="--config $c --steps 5 --warmup 1 --no-cpu-baseline --no-e2e"
  step ${c}_kt 240 rocprofv3 --kernel-trace --stats -d $OUT/${c}_kt -o run --output-format csv -- python3 bench.py $B
  tail -1 $OUT/${c}_kt.log > $OUT/bench_${c}_under_rocprof.json
  step ${c}_fetch 240 rocprofv3 --pmc FETCH_SIZE -d $OUT/${c}_fetch -o run --output-format csv -- python3 bench.py $B
  step ${c}_write 240 rocprofv3 --pmc WRITE_SIZE -d $OUT/${c}_write -o run --output-format csv -- python3 bench.py $B
  step ${c}_tcc 240 rocprofv3 --pmc TCC_EA0_ATOMIC_sum TCC_HIT_sum TCC_MISS_sum -d $OUT/${c}_tcc -o run --output-format csv -- python3 bench.py $B
  step ${c}_sq 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INSTS_VALU -d $OUT/${c}_sq -o run --output-format csv -- python3 bench.py $B
done
# C5 with the map adds compiled out (results wrong on purpose: cost split only)
XE_JIT_DEFINES=-DXE_DEBUG_NO_ATOMIC=1 step c5_noatomic 240 python3 bench.py --config c5 --steps 5 --warmup 1 --no-cpu-baseline --no-e2e
for k in 1 2 3; do
  step c3_rep$k 240 python3 bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline --no-e2e
done
echo done
