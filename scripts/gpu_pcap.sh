#!/bin/bash
# GPU check of the capture ingestion path: its parity test, then the pcap streaming rate for C2/C3.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; OUT=gpurun_out/pcap; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_xsk.py tests/test_c_example.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
for c in c2 c3; do
  timeout -k 10 300 python -u scripts/pcap_rate.py --config $c --packets 8388608 > $OUT/rate_$c.log 2>&1 || { tail -20 $OUT/rate_$c.log; exit 1; }
  tail -1 $OUT/rate_$c.log
done
