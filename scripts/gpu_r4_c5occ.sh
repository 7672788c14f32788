#!/bin/bash
# C5 occupancy A/B (tuning build): waves per SIMD the per-program kernel is compiled for
# (XE_JIT_DEFINES=-DXE_MIN_WAVES_PER_EU=w) and the persistent grid's blocks (XE_MAX_BLOCKS, 256 CUs).
# The product kernel is 4 waves/SIMD (126 VGPRs), 4 blocks (16 waves) per CU.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/r4c5occ; mkdir -p $OUT
export XE_LIB=$PWD/gobpfld_amd/libxdpemu_tuning.so
run() {  # tag waves blocks
  XE_JIT_DEFINES="-DXE_MIN_WAVES_PER_EU=$2" XE_MAX_BLOCKS=$3 timeout -k 10 240 python bench.py --config c5 --steps 8 \
    --no-e2e --no-cpu-baseline --no-verify > $OUT/$1.json 2>&1 || return 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], d['config'].get('grid'), r['avg_kernel_ms'], r['frac'])" $OUT/$1.json $1
}
run w4_b1024 4 1024 && run w5_b1280 5 1280 && run w4_b1280 4 1280 && run w6_b1280 6 1280
