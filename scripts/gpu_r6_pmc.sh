#!/bin/bash
# Round-6 PMC passes on the round-6 kernels (one counter group per rocprofv3 run, each under its own
# limit): FETCH_SIZE, WRITE_SIZE and TCC_EA0 read / atomic requests of C2, C3, C4 and C5 at bench size
# (each config alone: the default bench's side lines off), and 8 SQ counters of C4 and C5.
#   scripts/traffic.py gpurun_out/r6pmc profiles/r6 c2 c3 c4 c5  ->  profiles/r6/<config>_traffic.json
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r6pmc}; mkdir -p $OUT
ONLY="--no-cpu-baseline --no-e2e --no-ordered --no-c3 --no-c4 --no-c5"
for cfg in ${CONFIGS:-"c2:16777216" "c3:16777216" "c4:16777216" "c5:33554432"}; do
  c=${cfg%%:*}; n=${cfg##*:}
  for grp in "FETCH_SIZE:fetch" "WRITE_SIZE:write" "TCC_EA0_RDREQ_sum TCC_EA0_ATOMIC_sum:rdreq"; do
    ctrs=${grp%%:*}; tag=${grp##*:}
    timeout -s KILL 150 rocprofv3 --pmc $ctrs -d $OUT/${c}_$tag -o run --output-format csv -- python3 bench.py --config $c --packets $n --steps 5 --warmup 1 $ONLY > $OUT/${c}_$tag.log 2>&1 || { echo "pmc $c $tag failed"; tail -3 $OUT/${c}_$tag.log; exit 1; }
    echo "$c $tag done"
  done
done
for cfg in ${SQ_CONFIGS:-"c4:16777216" "c5:33554432"}; do
  c=${cfg%%:*}; n=${cfg##*:}
  timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY -d $OUT/${c}_sq -o run --output-format csv -- python3 bench.py --config $c --packets $n --steps 3 --warmup 1 $ONLY > $OUT/${c}_sq.log 2>&1 || { tail -3 $OUT/${c}_sq.log; exit 1; }
  echo "$c sq done"
done
