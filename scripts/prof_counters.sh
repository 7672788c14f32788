set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof1
export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/prof1/counters.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1/kt -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof1/bench_kt.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY -d gpurun_out/prof1/pmc1 -o run --output-format csv -- python3 bench.py --packets 2097152 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof1/pmc1.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d gpurun_out/prof1/pmc2 -o run --output-format csv -- python3 bench.py --packets 2097152 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof1/pmc2.log 2>&1 || exit 3
echo done
