#!/bin/bash
# Round 5: host-side marks of consecutive keyed batches (tuning build, XE_HOST_TIMING / XE_KEYED_TRACE)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5ks}; mkdir -p $OUT
export XE_LIB=$PWD/gobpfld_amd/libxdpemu_tuning.so XE_HOST_TIMING=1 XE_KEYED_TRACE=1
for c in c3learn c3lru; do
  timeout -k 10 300 python scripts/prof_keyed_stream.py $c 3 > $OUT/$c.log 2>&1 || { echo "$c failed"; tail -5 $OUT/$c.log; exit 1; }
  grep -E "^batch|host " $OUT/$c.log | tail -40
done
