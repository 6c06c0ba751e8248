#!/bin/bash
# round 6: config-3 packed pack by ticket items with the meta waves helping -- parity, A/B
set -u
export TMPDIR=/tmp
OUT=gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_pack_layout.py tests/test_gpu_pack_msgs.py tests/test_gpu_parity.py tests/test_gpu_tcp_tx.py \
  > $OUT/r06_s9_tests.log 2>&1 || { tail -40 $OUT/r06_s9_tests.log; exit 1; }
tail -3 $OUT/r06_s9_tests.log
timeout -k 10 600 bash scripts/ab_pack.sh || exit 1
