#!/bin/bash
# Why a keyed batch falls back on the device: the tuning build's XE_KEYED_TRACE lines for one case.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/diagk; mkdir -p $OUT
XE_LIB=$PWD/gobpfld_amd/libxdpemu_tuning.so XE_KEYED_TRACE=1 timeout -k 10 300 python -u -m pytest tests/test_ordered_par.py \
  -k "device_equal_oracle and lru_learn" -v -s --timeout 250 --timeout-method thread > $OUT/lru_learn.log 2>&1
echo "rc=$?"; grep -E "keyed:|PASS|FAIL|^E " $OUT/lru_learn.log | sort | uniq -c | head -30
