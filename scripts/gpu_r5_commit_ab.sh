#!/bin/bash
# Round 5: the committer wave (XE_COMMITTER) against the default kernel on the tuning build, C5 / C2 / bpf2bpf
# (the programs with paired adds) — every line verified against the header truth
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5commit}; mkdir -p $OUT
export XE_LIB=$PWD/gobpfld_amd/libxdpemu_tuning.so
run() {  # name config env...
  local name=$1 cfg=$2; shift 2
  env "$@" timeout -k 10 240 python bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-ordered --no-c5 --no-c4 > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; tail -3 $OUT/$name.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], d['value'], r['avg_kernel_ms'], d['verified'], d['config']['mode'])" $OUT/$name.json $name
}
run c5_base c5 XE_NONE=1 || exit 1
run c5_commit c5 XE_JIT_DEFINES=-DXE_COMMITTER=1 || exit 1
run c3_base c3 XE_NONE=1 || exit 1
run c3_commit c3 XE_JIT_DEFINES=-DXE_COMMITTER=1 || exit 1
run bpf_base bpf2bpf XE_NONE=1 || exit 1
run bpf_commit bpf2bpf XE_JIT_DEFINES=-DXE_COMMITTER=1 || exit 1
echo done
