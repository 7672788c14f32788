#!/bin/bash
# A/B of per-program kernel compile-time defines through the tuning build (XE_JIT_DEFINES), one bench
# process per variant, each under its own limit. Usage: gpu_ab.sh TAG "cfg[:packets]" "defines" ...
set -o pipefail
OUT=gpurun_out/$1; shift; mkdir -p $OUT
CFGS=$1; shift
export XE_LIB=$PWD/gobpfld_amd/libxdpemu_tuning.so
for cfg in $CFGS; do
  c=${cfg%%:*}; p=${cfg#*:}; [ "$p" = "$cfg" ] && p=0
  i=0
  for defs in "$@"; do
    i=$((i+1))
    XE_JIT_DEFINES="$defs" timeout -k 10 300 python bench.py --config $c --packets $p --no-cpu-baseline --no-e2e --no-ordered > $OUT/${c}_$i.json 2> $OUT/${c}_$i.err || { tail -5 $OUT/${c}_$i.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], repr(sys.argv[3]), d['value'], 'Mpkt/s kernel', r['avg_kernel_ms'], 'frac', r['frac'])" $OUT/${c}_$i.json $c "$defs"
  done
done
