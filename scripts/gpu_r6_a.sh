#!/bin/bash
# Round 6, first GPU call: the whole -m gpu suite (scripts/gpu_r6_suite.sh) on the in-tree build.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
TAG=r6a/suite bash scripts/gpu_r6_suite.sh
