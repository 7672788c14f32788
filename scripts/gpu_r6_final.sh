#!/bin/bash
# Round 6 close: the whole -m gpu suite, smoke(), then the default bench line and per-config kernel
# stats (scripts/gpu_r6_bench.sh), all on the in-tree build and kernel cache.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
T=${TAG:-r6final}
TAG=$T/suite bash scripts/gpu_r6_suite.sh || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.log 2>&1 || { tail -5 gpurun_out/$T/smoke.log; exit 1; }
tail -1 gpurun_out/$T/smoke.log
TAG=$T/bench bash scripts/gpu_r6_bench.sh
