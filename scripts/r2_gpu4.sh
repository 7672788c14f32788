#!/bin/bash
# Round 2, GPU call 4: C5 memory-shape calibration (tools/calib_hash) and the C3 placement
# experiment with map-buffer addresses (tuning library, XE_PRINT_ALLOC), default and 16 replicas.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/r2g4; mkdir -p $OUT
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $OUT/$name.log 2> $OUT/$name.err
  local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -25 $OUT/$name.log $OUT/$name.err; exit 1; }
}
step calib_hash 120 ./tools/calib_hash
cat $OUT/calib_hash.log
export XE_LIB=gobpfld_amd/libxdpemu_tuning.so XE_PRINT_ALLOC=1
step c3_place 400 python -u scripts/c3_placement2.py 16777216 10
cat $OUT/c3_place.log
XE_NREP=16 step c3_place_nrep16 300 python -u scripts/c3_placement2.py 16777216 6
cat $OUT/c3_place_nrep16.log
echo done
