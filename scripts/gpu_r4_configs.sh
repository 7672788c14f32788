#!/bin/bash
# Round 4: one bench line per config (each under its own limit), then rocprofv3 kernel stats of the
# default (C2) line and of bpf2bpf, and the PMC passes (one counter group per run) for C2 / C4f / C3 / C5.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/r4cfg; mkdir -p $OUT
B="--no-cpu-baseline --no-e2e"
line() {  # name args...
  local n=$1; shift
  timeout -k 10 240 python bench.py "$@" > $OUT/bench_$n.json 2> $OUT/bench_$n.err || { echo "bench $n failed"; tail -5 $OUT/bench_$n.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d.get('roofline',{}); print(sys.argv[2], d['value'], d['unit'], r.get('avg_kernel_ms'), r.get('frac'), d.get('verified'))" $OUT/bench_$n.json $n
}
[ -n "$LINES" ] && { line c3 --config c3 $B --no-ordered && line c4 --config c4 $B --no-ordered && line c4f --config c4f $B --no-ordered &&
line c5 --config c5 $B --no-ordered && line bpf2bpf --config bpf2bpf $B --no-ordered && line c1 --config c1 $B --no-ordered || exit 1; }
timeout -k 10 400 python -u -m pytest tests/test_ordered_par.py -m gpu -v --maxfail=5 --timeout 200 --timeout-method thread > $OUT/pytest_ordered.log 2>&1; rc=$?
tail -2 $OUT/pytest_ordered.log; [ $rc -eq 0 ] || { grep -E "FAILED|^E " $OUT/pytest_ordered.log | head; exit 1; }
timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d $OUT/prof_c2 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 $B --no-ordered --no-c5 > $OUT/prof_c2.log 2>&1 || { echo "prof c2 failed"; tail -3 $OUT/prof_c2.log; exit 1; }
timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d $OUT/prof_bpf2bpf -o run --output-format csv -- python3 bench.py --config bpf2bpf --steps 10 --warmup 2 $B --no-ordered > $OUT/prof_bpf2bpf.log 2>&1 || { echo "prof bpf2bpf failed"; tail -3 $OUT/prof_bpf2bpf.log; exit 1; }
echo "kernel stats done"
for cfg in "c2 16777216" "c4f 16777216" "c3 16777216" "c5 33554432"; do
  set -- $cfg
  for grp in "FETCH_SIZE:fetch" "WRITE_SIZE:write" "TCC_EA0_RDREQ_sum TCC_EA0_ATOMIC_sum:rdreq"; do
    ctrs=${grp%%:*}; tag=${grp##*:}
    timeout -s KILL 120 rocprofv3 --pmc $ctrs -d $OUT/${1}_$tag -o run --output-format csv -- python3 bench.py --config $1 --packets $2 --steps 5 --warmup 1 $B --no-ordered --no-c5 --no-verify > $OUT/${1}_$tag.log 2>&1 || { echo "pmc $1 $tag failed"; tail -3 $OUT/${1}_$tag.log; exit 1; }
  done
  echo "$1 pmc done"
done
for c in c2 c5; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY -d $OUT/${c}_sq -o run --output-format csv -- python3 bench.py --config $c --steps 3 --warmup 1 $B --no-ordered --no-c5 --no-verify > $OUT/${c}_sq.log 2>&1 || { echo "sq $c failed"; tail -3 $OUT/${c}_sq.log; exit 1; }
done
echo "all done"
