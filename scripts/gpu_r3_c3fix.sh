#!/bin/bash
# C3 modes on the product (16 replicas, sparse fold), then the suite, smoke and the C1-C5 lines.
set -o pipefail
T=${1:-r3g}
bash scripts/c3_modes.sh ${T}_c3modes || exit 1
bash scripts/gpu_r3_suite.sh $T && bash scripts/gpu_r3_configs.sh $T || exit 1
