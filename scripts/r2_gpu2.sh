#!/bin/bash
# Round 2, GPU call 2: grouped hash probing (one burst load per 128-B record group). Parity suite on
# the product library, then C5/C3 kernel time for probe groups 0 (one record per round trip) / 64 / 128
# through the tuning library.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/r2g2; mkdir -p $OUT
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -25 $OUT/$name.log; exit 1; }
}
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
tail -1 $OUT/pytest_gpu.log
for c in c5 c3; do
  for g in 0 64 128 0 128; do
    XE_LIB=gobpfld_amd/libxdpemu_tuning.so XE_JIT_DEFINES=-DXE_PROBE_GROUP=$g step ${c}_g$g 240 python bench.py --config $c --steps 6 --warmup 2 --no-cpu-baseline --no-e2e
    grep -o '"avg_kernel_ms": [0-9.]*' $OUT/${c}_g$g.log | sed "s/^/$c group $g /"
  done
done
echo done
