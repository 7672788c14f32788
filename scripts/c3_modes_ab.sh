#!/bin/bash
# C3 run-to-run modes with the tuning build's replica knob (XE_NREP): ten fresh processes per setting.
set -o pipefail
OUT=gpurun_out/${1:-c3modes_ab}; mkdir -p $OUT
export XE_LIB=$PWD/gobpfld_amd/libxdpemu_tuning.so
for nrep in ${NREPS:-16 4}; do
  for i in 1 2 3 4 5 6 7 8 9 10; do
    XE_NREP=$nrep timeout -k 10 240 python bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-ordered > $OUT/c3_n${nrep}_$i.json 2> $OUT/c3_n${nrep}_$i.err || { tail -5 $OUT/c3_n${nrep}_$i.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('nrep', sys.argv[3], 'run', sys.argv[2], d['value'], 'Mpkt/s kernel', d['roofline']['avg_kernel_ms'], 'step', d['ms_per_step'])" $OUT/c3_n${nrep}_$i.json $i $nrep
  done
done
