#!/bin/bash
# Round 5: what the one-lane in-order replay spends its time on (C2-RMW, C3-learn, C3-LRU at 65,536 packets):
# kernel time per packet and the SQ counters of the replay kernel; then the runahead A/B (tuning build,
# XE_SEQ_PEEK=0 / 1)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5seq}; mkdir -p $OUT
show() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['roofline']['avg_kernel_ms'], d['config']['mode'], d['config']['insns_per_packet'])" "$@"; }
for c in ${CONFIGS:-c2rmw c3learn c3lru c3lrufull}; do
  B="--config $c --packets 65536 --mode sequential --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-ordered --no-c5 --no-c4 --no-verify --sync"
  timeout -k 10 240 python bench.py $B > $OUT/$c.json 2> $OUT/$c.err || { echo "$c failed"; tail -3 $OUT/$c.err; exit 1; }
  show $OUT/$c.json $c
  [ -n "$NO_SQ" ] || { timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY -d $OUT/${c}_sq -o run --output-format csv -- python3 bench.py $B > $OUT/${c}_sq.log 2>&1 || { echo "sq $c failed"; tail -3 $OUT/${c}_sq.log; exit 1; }; }
  [ -n "$AB" ] && for pk in 0 1; do
    XE_LIB=$PWD/gobpfld_amd/libxdpemu_tuning.so XE_SEQ_PEEK=$pk timeout -k 10 240 python bench.py $B > $OUT/${c}_peek$pk.json 2> $OUT/${c}_peek$pk.err || { echo "$c peek $pk failed"; tail -3 $OUT/${c}_peek$pk.err; exit 1; }
    show $OUT/${c}_peek$pk.json "$c peek=$pk"
  done
done
find $OUT -name "*.db" -delete; du -sh $OUT; echo done
