#!/bin/bash
# Round 6: rule-chain dispatch (xe_jit.cpp rule_chain_at): its parity tests and the tests that run C4 /
# branchy programs on the device, then the C4 line on the product build under rocprofv3 --kernel-trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r6rc}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_rule_chain.py tests/test_segments.py \
  tests/test_wave_steps.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_c4 -o run -- python3 bench.py --config c4 --no-cpu-baseline --no-e2e > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { tail -5 $OUT/bench_c4.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print('c4', d['value'], d['ms_per_step'], r['avg_kernel_ms'], r['frac'], d.get('verified'))" $OUT/bench_c4.json
