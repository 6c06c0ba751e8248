#!/bin/bash
set -u
export TMPDIR=/tmp
OUT=gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_analytics.py tests/test_gpu_worker.py > $OUT/r06_s5_tests.log 2>&1 || { tail -40 $OUT/r06_s5_tests.log; exit 1; }
tail -3 $OUT/r06_s5_tests.log
timeout -k 10 600 bash scripts/ab_c4.sh || exit 1
timeout -k 10 300 python3 scripts/skel_prof.py || exit 1
