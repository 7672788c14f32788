#!/bin/bash
# counter comparison across configs (JIT engine); one PMC group per pass
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; OUT=gpurun_out/cmp; mkdir -p $OUT
for cfg in c1:16777216 c2:4194304 c4:1048576 c4:8388608; do
  name=${cfg%%:*}; n=${cfg##*:}
  i=0
  for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_IFETCH" "SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_INSTS_FLAT SQ_WAIT_INST_LDS"; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --pmc $grp -d $OUT/${name}_${n}_$i -o run --output-format csv -- python3 bench.py --config $name --packets $n --steps 2 --warmup 1 --engine jit --no-cpu-baseline > $OUT/${name}_${n}_$i.log 2>&1 || { echo "fail $name $i"; tail -3 $OUT/${name}_${n}_$i.log; exit 1; }
  done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/${name}_${n}_kt -o run --output-format csv -- python3 bench.py --config $name --packets $n --steps 3 --warmup 1 --engine jit --no-cpu-baseline > $OUT/${name}_${n}_kt.log 2>&1 || exit 1
done
echo done
