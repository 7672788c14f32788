#!/bin/bash
# Round 5: per-dispatch kernel trace of a stream of keyed batches on one VM (product build):
# which passes a steady keyed batch spends its device time in.  CONFIGS="c3lru c3learn" by default.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5kp}; mkdir -p $OUT
for c in ${CONFIGS:-c3lru c3learn}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$c -o run --output-format csv -- python3 scripts/prof_keyed_stream.py $c ${BATCHES:-4} > $OUT/$c.log 2>&1 || { echo "$c failed"; tail -5 $OUT/$c.log; exit 1; }
  grep -E "^batch" $OUT/$c.log
done
find $OUT -name '*.db' -delete
du -sh $OUT
