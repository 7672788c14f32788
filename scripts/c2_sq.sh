#!/bin/bash
# C2 issue-side counters (one --pmc pass, 8 SQ counters) and the bench line of the same tree.
set -e
OUT=gpurun_out/c2sq
mkdir -p $OUT
timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --no-ordered > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU -d $OUT/pmc -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-ordered > $OUT/pmc.log 2>&1 || { tail -5 $OUT/pmc.log; exit 1; }
echo ok
