#!/bin/bash
# Keyed C3-LRU host-side timeline (tuning build, XE_HOST_TIMING marks per batch)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/r4lruh; mkdir -p $OUT
XE_LIB=$PWD/gobpfld_amd/libxdpemu_tuning.so XE_HOST_TIMING=1 timeout -k 10 300 python3 scripts/prof_c3lru.py > $OUT/host.log 2>&1 || { tail -5 $OUT/host.log; exit 1; }
grep -v "n=0)" $OUT/host.log | tail -40
