#!/bin/bash
# round 6: FindFlow row keys in two loads; TCP records by ticket with the meta waves helping
set -u
export TMPDIR=/tmp
OUT=gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_flowtab.py tests/test_gpu_tcp_tx.py tests/test_gpu_scan.py \
  > $OUT/r06_s8_tests.log 2>&1 || { tail -40 $OUT/r06_s8_tests.log; exit 1; }
tail -3 $OUT/r06_s8_tests.log
timeout -k 10 300 python3 scripts/ft_time.py || exit 1
timeout -k 10 300 python3 scripts/ft_time.py || exit 1
timeout -k 10 600 bash scripts/ab_tcp.sh || exit 1
