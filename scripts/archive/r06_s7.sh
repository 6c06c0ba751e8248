#!/bin/bash
# round 6: the restored one-wave-per-flow update (parity + A/B), then config-3 counters
set -u
export TMPDIR=/tmp
OUT=gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_analytics.py > $OUT/r06_s7_tests.log 2>&1 || { tail -40 $OUT/r06_s7_tests.log; exit 1; }
tail -3 $OUT/r06_s7_tests.log
timeout -k 10 600 bash scripts/ab_c4.sh || exit 1
ROUND=r06 timeout -k 10 900 bash scripts/pmc_c3.sh || exit 1
cat $OUT/traffic_config3.json
