#!/bin/bash
# Round-3 PMC passes (one counter group per rocprofv3 run, each under its own limit): FETCH_SIZE,
# WRITE_SIZE and TCC_EA0 read / atomic requests of C2-C5 at bench size, and the C2 SQ issue counters.
set -o pipefail
T=${1:-r3pmc}
OUT=gpurun_out/$T; mkdir -p $OUT
export TMPDIR=/tmp
for cfg in "c2 16777216" "c3 16777216" "c4 16777216" "c5 33554432"; do
  set -- $cfg
  for grp in "FETCH_SIZE:fetch" "WRITE_SIZE:write" "TCC_EA0_RDREQ_sum TCC_EA0_ATOMIC_sum:rdreq"; do
    ctrs=${grp%%:*}; tag=${grp##*:}
    timeout -s KILL 120 rocprofv3 --pmc $ctrs -d $OUT/${1}_$tag -o run --output-format csv -- python3 bench.py --config $1 --packets $2 --steps 5 --warmup 1 --no-cpu-baseline --no-e2e --no-ordered > $OUT/${1}_$tag.log 2>&1 || { echo "pmc $1 $tag failed"; tail -3 $OUT/${1}_$tag.log; exit 1; }
    echo "$1 $tag done"
  done
done
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU -d $OUT/c2_sq -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-ordered > $OUT/c2_sq.log 2>&1 || { tail -3 $OUT/c2_sq.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY -d $OUT/c5_sq -o run --output-format csv -- python3 bench.py --config c5 --packets 33554432 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-ordered > $OUT/c5_sq.log 2>&1 || { tail -3 $OUT/c5_sq.log; exit 1; }
echo "sq done"
