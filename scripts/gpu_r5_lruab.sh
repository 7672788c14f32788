#!/bin/bash
# Round 5: what the keyed C3-LRU passes spend their time on (tuning build, XE_JIT_DEFINES, one box):
# the default kernel, LRU touches dropped, map adds dropped, both (results wrong in the variants)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5lruab}; mkdir -p $OUT
export XE_LIB=$PWD/gobpfld_amd/libxdpemu_tuning.so
for d in "" "-DXE_DEBUG_NO_LRU_TOUCH" "-DXE_DEBUG_NO_ATOMIC" "-DXE_DEBUG_NO_LRU_TOUCH -DXE_DEBUG_NO_ATOMIC"; do
  XE_JIT_DEFINES="$d" timeout -k 10 300 python scripts/prof_keyed_stream.py c3lru 4 > $OUT/ab.log 2>&1 || { echo "$d failed"; tail -3 $OUT/ab.log; exit 1; }
  echo "defines [$d]: $(grep '^batch' $OUT/ab.log | tail -3 | tr '\n' ' ')"
done
