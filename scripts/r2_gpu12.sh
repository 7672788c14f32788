#!/bin/bash
# Round 2, GPU call 12: where the C2 kernel's time goes (SQ pass) on the deferred-commit tree, and
# C2 at 3 resident blocks per CU; C5 cost split (probe / adds compiled out, tuning build).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/r2g12; mkdir -p $OUT
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  timeout -k 10 -s KILL $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -15 $OUT/$name.log; exit 1; }
}
B="--steps 5 --warmup 1 --no-cpu-baseline --no-e2e --no-ordered --sync"
step c2_sq 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INSTS_VALU -d $OUT/c2_sq -o run --output-format csv -- python3 bench.py $B
step c2_sq2 240 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_WAVE_CYCLES -d $OUT/c2_sq2 -o run --output-format csv -- python3 bench.py $B
step c5_sq 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INSTS_VALU -d $OUT/c5_sq -o run --output-format csv -- python3 bench.py --config c5 $B
XE_LIB=gobpfld_amd/libxdpemu_tuning.so XE_MAX_BLOCKS=768 step c2_g768 240 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-ordered
grep -o '"value": [0-9.]*\|"avg_kernel_ms": [0-9.]*' $OUT/c2_g768.log | tr '\n' ' '; echo
T="XE_LIB=gobpfld_amd/libxdpemu_tuning.so"
for d in "-DXE_DEBUG_NO_PROBE=1" "-DXE_DEBUG_NO_ATOMIC=1" "-DXE_DEBUG_NO_PROBE=1 -DXE_DEBUG_NO_ATOMIC=1"; do
  n=c5$(echo $d | tr -d ' =' | tr 'A-Z' 'a-z' | sed 's/-dxe_debug_//g')
  XE_LIB=gobpfld_amd/libxdpemu_tuning.so XE_JIT_DEFINES="$d" step $n 240 python bench.py --config c5 --steps 6 --warmup 2 --no-cpu-baseline --no-e2e
  grep -o '"avg_kernel_ms": [0-9.]*' $OUT/$n.log
done
echo done
