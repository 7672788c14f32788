#!/bin/bash
# Round 4, third pass: why lru_learn_queue falls back on the device (tuning build trace), smoke(), the
# default bench line, one line per config.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
bash scripts/gpu_diag_keyed.sh
OUT=gpurun_out/r4b3; mkdir -p $OUT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && tail -1 $OUT/smoke.log &&
timeout -k 10 420 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err && echo bench ok && tail -c 1500 $OUT/bench_default.json || { tail -20 $OUT/bench_default.err; exit 1; }
B="--no-cpu-baseline --no-e2e --no-ordered"
line() {  # name args...
  local n=$1; shift
  timeout -k 10 240 python bench.py "$@" > $OUT/bench_$n.json 2> $OUT/bench_$n.err || { echo "bench $n failed"; tail -5 $OUT/bench_$n.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d.get('roofline',{}); print(sys.argv[2], d['value'], d['unit'], r.get('avg_kernel_ms'), r.get('frac'), d.get('verified'))" $OUT/bench_$n.json $n
}
line c3 --config c3 $B && line c4 --config c4 $B && line c4f --config c4f $B && line c5 --config c5 $B &&
line bpf2bpf --config bpf2bpf $B && line c1 --config c1 $B
