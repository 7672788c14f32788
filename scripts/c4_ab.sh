#!/bin/bash
# A/B on one box (tuning library, XE_JIT_DEFINES): C4 and C2 kernel times with the one-ballot status
# histogram and the skip-mask check on / off.
set -e
OUT=gpurun_out/c4ab
mkdir -p $OUT
export XE_LIB=$GRAFT_REPO_ROOT/gobpfld_amd/libxdpemu_tuning.so
for cfg in c4 c2; do
  for d in "" "-DXE_HIST_FAST=0" "-DXE_SKIP_MASK=0" "-DXE_HIST_FAST=0 -DXE_SKIP_MASK=0" ""; do
    XE_JIT_DEFINES="$d" timeout -k 10 200 python bench.py --config $cfg --no-cpu-baseline --no-e2e --no-ordered --steps 10 > $OUT/b.json 2> $OUT/b.err || { tail -3 $OUT/b.err; exit 1; }
    python3 -c "import json; b=json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); print('$cfg', '[$d]', b['roofline']['avg_kernel_ms'])" | tee -a $OUT/ab.txt
  done
done
