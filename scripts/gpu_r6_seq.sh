#!/bin/bash
# Round 6: the one-lane replay under rocprofv3 — kernel trace (which variant ran: VGPR / SGPR counts)
# and one pass of 8 SQ counters per config (per-packet instruction mix).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r6seq}; mkdir -p $OUT
for c in ${CONFIGS:-c2rmw c3learn c3lru}; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/kt_$c -o run --output-format csv -- python3 scripts/prof_seq.py $c 65536 2 > $OUT/kt_$c.log 2>&1 || { tail -5 $OUT/kt_$c.log; exit 1; }
  cat $OUT/kt_$c.log | grep run
  timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY -d $OUT/sq_$c -o run --output-format csv -- python3 scripts/prof_seq.py $c 65536 1 > $OUT/sq_$c.log 2>&1 || { tail -5 $OUT/sq_$c.log; exit 1; }
done
