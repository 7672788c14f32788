#!/bin/bash
# Round 5 A/B through the tuning build's XE_JIT_DEFINES (per-program kernel -D options): C4 with and
# without if-converted jump blocks, C4 / C2 with and without the one-lane runahead's gates compiled in
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5ab}; mkdir -p $OUT
B="--no-cpu-baseline --no-e2e --no-ordered --no-c5 --no-c4 --no-verify"
export XE_LIB=$PWD/gobpfld_amd/libxdpemu_tuning.so
for c in ${CONFIGS:-c4 c2}; do
  for d in "-DXE_IFCONV=0" "-DXE_IFCONV=1" "-DXE_IFCONV=0 -DXE_SEQ_PEEK=0"; do
    XE_JIT_DEFINES="$d" timeout -k 10 300 python bench.py --config $c $B > $OUT/ab.json 2> $OUT/ab.err || { echo "$c $d failed"; tail -3 $OUT/ab.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['roofline']['avg_kernel_ms'])" $OUT/ab.json "$c $d"
  done
done
