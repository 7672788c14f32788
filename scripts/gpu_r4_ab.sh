#!/bin/bash
# Round-4 A/B (tuning build): C5 occupancy (waves per SIMD the kernel is compiled for, XE_MIN_WAVES_PER_EU,
# and the persistent grid, XE_MAX_BLOCKS over 256 CUs) and C3's per-wave accumulator size (XE_ACC).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/r4ab; mkdir -p $OUT
export XE_LIB=$PWD/gobpfld_amd/libxdpemu_tuning.so
run() {  # tag config defines blocks
  XE_JIT_DEFINES="$3" XE_MAX_BLOCKS=$4 timeout -k 10 240 python bench.py --config $2 --steps 8 --no-e2e --no-cpu-baseline \
    --no-ordered --no-verify > $OUT/$1.json 2> $OUT/$1.err || { tail -3 $OUT/$1.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], d['config'].get('grid'), r['avg_kernel_ms'], r['frac'])" $OUT/$1.json $1
}
run c5_w4_b1024 c5 "-DXE_MIN_WAVES_PER_EU=4" 1024 && run c5_w5_b1280 c5 "-DXE_MIN_WAVES_PER_EU=5" 1280 &&
run c5_w6_b1536 c5 "-DXE_MIN_WAVES_PER_EU=6" 1536 &&
run c3_acc64 c3 "-DXE_ACC=64" 1024 && run c3_acc128 c3 "-DXE_ACC=128" 1024 && run c3_acc256 c3 "-DXE_ACC=256" 1024
