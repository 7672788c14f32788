#!/bin/bash
# Profiles of the bench command (default C2 JIT): kernel trace + stats, then one PMC pass per counter group.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/${PROF_TAG:-prof}; mkdir -p $OUT
ARGS=${BENCH_ARGS:-"--steps 10 --warmup 2 --no-cpu-baseline"}
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python3 bench.py $ARGS > $OUT/bench_kt.log 2>&1 || exit 1
tail -1 $OUT/bench_kt.log > $OUT/bench_line.json
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH" "TCP_TOTAL_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 400 rocprofv3 --pmc $grp -d $OUT/pmc$i -o run --output-format csv -- python3 bench.py $ARGS --steps 3 --warmup 1 > $OUT/pmc$i.log 2>&1 || { echo "pmc group $i failed"; tail -3 $OUT/pmc$i.log; }
done
echo done
