#!/bin/bash
# Grid A/B: resident blocks per CU for each config (tuning build, XE_MAX_BLOCKS caps the persistent grid).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/r4grid; mkdir -p $OUT
export XE_LIB=$PWD/gobpfld_amd/libxdpemu_tuning.so
run() {  # cfg blocks
  XE_MAX_BLOCKS=$2 timeout -k 10 150 python bench.py --config $1 --no-c5 --no-ordered --no-e2e --no-cpu-baseline --no-verify > $OUT/$1_mb$2.json 2>&1 || return 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], sys.argv[3], d['config']['grid'], r['avg_kernel_ms'], r['frac'])" $OUT/$1_mb$2.json $1 $2
}
for mb in 512 768 1024 99999; do run c2 $mb || exit 1; done
for mb in 512 768 1024 99999; do run c4 $mb || exit 1; done
for mb in 768 1024 99999; do run c3 $mb || exit 1; done
for mb in 512 768 1024 99999; do run c5 $mb || exit 1; done
