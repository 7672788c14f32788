#!/bin/bash
# Round 6: what the dependent hash probe costs C5 and C3 (the bound on a probe prefetch): the default
# kernel, the probe compiled out (every key hits its home slot: XE_DEBUG_NO_PROBE, wrong results, verify
# off), and both the probe and the map adds out; tuning build, one bench process per variant
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r6probe}; mkdir -p $OUT
export XE_LIB=$PWD/gobpfld_amd/libxdpemu_tuning.so
run() {  # name, config, defines, extra args
  local name=$1 cfg=$2 defs=$3; shift 3
  XE_JIT_DEFINES="$defs" timeout -k 10 240 python bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline --no-e2e \
    --no-ordered --no-c5 --no-c4 --no-c3 "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; tail -3 $OUT/$name.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], d['value'], r['avg_kernel_ms'], d['verified'])" $OUT/$name.json $name
}
run c5_base c5 "" || exit 1
run c5_noprobe c5 "-DXE_DEBUG_NO_PROBE" --no-verify || exit 1
run c5_noprobe_noatomic c5 "-DXE_DEBUG_NO_PROBE -DXE_DEBUG_NO_ATOMIC" --no-verify || exit 1
run c3_base c3 "" || exit 1
run c3_noprobe c3 "-DXE_DEBUG_NO_PROBE" --no-verify || exit 1
echo done
