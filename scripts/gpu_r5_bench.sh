#!/bin/bash
# Round 5 measurements. PART=a: the default bench line (C2 + C5 / C4 side lines + ordered / keyed lines), its
# C2 kernel stats, and C1 / C3 / C4f / bpf2bpf lines. PART=b: C4 / C5 / bpf2bpf kernel stats, C4 / C5 SQ counter
# passes and PMC traffic passes (one counter group per run).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5bench}; mkdir -p $OUT
B="--no-cpu-baseline --no-e2e --no-ordered --no-c5 --no-c4"
if [ "${PART:-a}" = a ]; then
  timeout -k 10 500 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('c2', d['value'], d['roofline']['frac'], d['verified']); print('c5', d['c5']['value'], d['c5']['avg_kernel_ms'], d['c5']['verified']); print('c4', d['c4']['value'], d['c4']['avg_kernel_ms'], d['c4']['verified']); o=d['ordered']; print({k: (o[k]['keyed']['value'], o[k]['keyed']['mode_used'], o[k]['sequential_one_lane']['value']) for k in o if k.startswith('keyed')})" $OUT/bench.json
  timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_c2 -o run --output-format csv -- python3 bench.py $B > $OUT/prof_c2.log 2>&1 || { echo "prof c2 failed"; tail -3 $OUT/prof_c2.log; exit 1; }
  for c in c1 c3 c4f bpf2bpf; do
    timeout -k 10 300 python bench.py --config $c $B > $OUT/bench_$c.json 2> $OUT/bench_$c.err || { echo "bench $c failed"; tail -3 $OUT/bench_$c.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['roofline']['avg_kernel_ms'], d['roofline']['frac'], d['verified'])" $OUT/bench_$c.json $c
  done
else
  for c in c4 c5; do
    timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$c -o run --output-format csv -- python3 bench.py --config $c --steps 10 --warmup 2 $B > $OUT/prof_$c.log 2>&1 || { echo "prof $c failed"; tail -3 $OUT/prof_$c.log; exit 1; }
    timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY -d $OUT/${c}_sq -o run --output-format csv -- python3 bench.py --config $c --steps 3 --warmup 1 $B --no-verify > $OUT/${c}_sq.log 2>&1 || { echo "sq $c failed"; tail -3 $OUT/${c}_sq.log; exit 1; }
    for grp in "FETCH_SIZE:fetch" "WRITE_SIZE:write" "TCC_EA0_RDREQ_sum TCC_EA0_ATOMIC_sum:rdreq"; do
      ctrs=${grp%%:*}; tag=${grp##*:}
      timeout -s KILL 150 rocprofv3 --pmc $ctrs -d $OUT/${c}_$tag -o run --output-format csv -- python3 bench.py --config $c --steps 5 --warmup 1 $B --no-verify > $OUT/${c}_$tag.log 2>&1 || { echo "pmc $c $tag failed"; tail -3 $OUT/${c}_$tag.log; exit 1; }
    done
    echo "$c profiled"
  done
  timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_bpf2bpf -o run --output-format csv -- python3 bench.py --config bpf2bpf --steps 10 --warmup 2 $B > $OUT/prof_bpf2bpf.log 2>&1 || { echo "prof bpf2bpf failed"; tail -3 $OUT/prof_bpf2bpf.log; exit 1; }
fi
find $OUT -name "*.db" -delete; du -sh $OUT; echo "all done"
