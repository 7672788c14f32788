#!/bin/bash
# Round-2 final bench evidence (after the keyed path): the default bench line, the kernel-trace
# statistics of the C2 steps alone (no ordered / keyed side lines, so the xe_jit_kernel average is the
# C2 kernel's), and the keyed C3-learn line at 16M packets.
set -e
OUT=gpurun_out/r2final2
mkdir -p $OUT
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-e2e --no-ordered > $OUT/bench_kt.json 2> $OUT/bench_kt.err || { tail -5 $OUT/bench_kt.err; exit 1; }
timeout -k 10 400 python3 -c "
import json, torch, bench
dev = torch.device('cuda', 0)
print(json.dumps(bench.keyed_paths(dev, torch.cuda.current_stream(dev).cuda_stream, 16777216, reps=3)))
" > $OUT/keyed_16M.json 2> $OUT/keyed_16M.err || { tail -5 $OUT/keyed_16M.err; exit 1; }
echo ok
