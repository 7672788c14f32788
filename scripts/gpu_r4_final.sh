#!/bin/bash
# Round 4 close: the key-shadow device tests (the rest of the -m gpu suite passed on this tree, gpu_r4_suite.sh),
# smoke(), the default bench line and the keyed C3-LRU profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/r4f; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_key_shadow.py -m gpu -v --timeout 200 --timeout-method thread > $OUT/pytest_ks.log 2>&1; rc=$?
tail -2 $OUT/pytest_ks.log; [ $rc -eq 0 ] || { grep -E "FAILED|^E " $OUT/pytest_ks.log | head -20; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && tail -1 $OUT/smoke.log &&
timeout -k 10 420 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err && echo bench ok || exit 1
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_c3lru -o run --output-format csv -- python3 scripts/prof_c3lru.py > $OUT/prof_c3lru.log 2>&1 || { echo "prof c3lru failed"; tail -3 $OUT/prof_c3lru.log; exit 1; }
grep keyed $OUT/prof_c3lru.log | tail -1
echo all done
