#!/bin/bash
# Round 5 C5 A/B on the tuning build: the default kernel, map adds compiled out, no deferred commit,
# a 4x sparser hash table (fewer probe groups left), one pass each (bench --config c5, verify off where
# the variant changes results)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5c5ab}; mkdir -p $OUT
export XE_LIB=$PWD/gobpfld_amd/libxdpemu_tuning.so
B="--config c5 --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-ordered --no-c5 --no-c4"
run() {  # name, env..., extra args
  local name=$1; shift
  env "$@" timeout -k 10 240 python bench.py $B $EXTRA > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; tail -3 $OUT/$name.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], d['value'], r['avg_kernel_ms'], d['verified'])" $OUT/$name.json $name
}
EXTRA="" run base XE_NONE=1 || exit 1
EXTRA="--no-verify" run noatomic XE_JIT_DEFINES=-DXE_DEBUG_NO_ATOMIC || exit 1
EXTRA="" run nodefer XE_JIT_DEFINES=-DXE_DEFER_COMMIT=0 || exit 1
EXTRA="" run capx4 XE_HASH_CAPX=4 || exit 1
EXTRA="" run capx8 XE_HASH_CAPX=8 || exit 1
echo done
