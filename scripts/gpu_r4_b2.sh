#!/bin/bash
# Round 4, second pass: the ordered-map device tests, smoke(), the default bench line and one line per config.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/r4b2; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_ordered_par.py tests/test_step_api.py -m gpu -v --maxfail=5 --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAILED|^E " $OUT/pytest_gpu.log | head -20; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && tail -1 $OUT/smoke.log &&
timeout -k 10 420 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err && echo bench ok && tail -c 600 $OUT/bench_default.json || exit 1
B="--no-cpu-baseline --no-e2e --no-ordered"
line() {  # name args...
  local n=$1; shift
  timeout -k 10 240 python bench.py "$@" > $OUT/bench_$n.json 2> $OUT/bench_$n.err || { echo "bench $n failed"; tail -5 $OUT/bench_$n.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d.get('roofline',{}); print(sys.argv[2], d['value'], d['unit'], r.get('avg_kernel_ms'), r.get('frac'), d.get('verified'))" $OUT/bench_$n.json $n
}
line c3 --config c3 $B && line c4 --config c4 $B && line c4f --config c4f $B && line c5 --config c5 $B &&
line bpf2bpf --config bpf2bpf $B && line c1 --config c1 $B
