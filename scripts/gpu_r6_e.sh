#!/bin/bash
# Round 6: the whole -m gpu suite, then C4 (lazily if-converted jump chains) timed and one SQ pass.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r6e}; mkdir -p $OUT
TAG=${TAG:-r6e}/suite bash scripts/gpu_r6_suite.sh || exit 1
ONLY="--no-cpu-baseline --no-e2e --no-ordered --no-c3 --no-c4 --no-c5"
timeout -k 10 300 python3 bench.py --config c4 --packets 16777216 --steps 20 --warmup 3 $ONLY > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { tail -5 $OUT/bench_c4.err; exit 1; }
cut -c1-300 $OUT/bench_c4.json
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY -d $OUT/c4_sq -o run --output-format csv -- python3 bench.py --config c4 --packets 16777216 --steps 3 --warmup 1 $ONLY > $OUT/c4_sq.log 2>&1 || { tail -3 $OUT/c4_sq.log; exit 1; }
echo done
