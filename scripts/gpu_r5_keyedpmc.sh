#!/bin/bash
# Round 5: SQ counters and memory-side atomics of the keyed passes (SPEC, parallel) of a keyed stream
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5kpmc}; mkdir -p $OUT
for c in ${CONFIGS:-c3lru c3learn}; do
  timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY -d $OUT/${c}_sq -o run --output-format csv -- python3 scripts/prof_keyed_stream.py $c 3 > $OUT/${c}_sq.log 2>&1 || { echo "sq $c failed"; tail -3 $OUT/${c}_sq.log; exit 1; }
  timeout -s KILL 150 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_ATOMIC_sum -d $OUT/${c}_rq -o run --output-format csv -- python3 scripts/prof_keyed_stream.py $c 3 > $OUT/${c}_rq.log 2>&1 || { echo "rq $c failed"; tail -3 $OUT/${c}_rq.log; exit 1; }
  echo "$c done"
done
find $OUT -name '*.db' -delete; du -sh $OUT
