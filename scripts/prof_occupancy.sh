#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/occ; export TMPDIR=/tmp
for cfg in "c1 16777216" "c2 4194304" "c4 1048576"; do
  set -- $cfg
  for eng in jit interp; do
    timeout -k 10 300 python bench.py --config $1 --packets $2 --steps 5 --warmup 1 --engine $eng --no-cpu-baseline > gpurun_out/occ/bench_${1}_${eng}.log 2>&1 || exit 1
    echo "$1 $eng $(tail -1 gpurun_out/occ/bench_${1}_${eng}.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], "Mpkt/s kernel_ms", d["roofline"]["avg_kernel_ms"], "insns", d["config"]["insns_per_packet"])')"
  done
done
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LEVEL_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAIT_ANY -d gpurun_out/occ/pmc_c2jit -o run --output-format csv -- python3 bench.py --config c2 --packets 4194304 --steps 2 --warmup 1 --engine jit --no-cpu-baseline > gpurun_out/occ/pmc_c2jit.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LEVEL_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAIT_ANY -d gpurun_out/occ/pmc_c4jit -o run --output-format csv -- python3 bench.py --config c4 --packets 1048576 --steps 2 --warmup 1 --engine jit --no-cpu-baseline > gpurun_out/occ/pmc_c4jit.log 2>&1 || exit 3
echo done
