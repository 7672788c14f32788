#!/bin/bash
# Suite + smoke + default bench, then the C1-C5 lines, then an optional A/B (ARGS for gpu_ab.sh).
set -o pipefail
T=${1:-r3}; shift
bash scripts/gpu_r3_suite.sh $T && bash scripts/gpu_r3_configs.sh $T || exit 1
if [ $# -gt 0 ]; then bash scripts/gpu_ab.sh ${T}_ab "$@" || exit 1; fi
