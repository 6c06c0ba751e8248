#!/bin/bash
# round 6: long-record unpack shapes (config 5) -- parity of the product shape, then the sweep
set -u
export TMPDIR=/tmp
OUT=gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_unpack_long.py > $OUT/r06_s13_tests.log 2>&1 || { tail -40 $OUT/r06_s13_tests.log; exit 1; }
tail -3 $OUT/r06_s13_tests.log
timeout -k 10 600 python3 -u scripts/c5_shapes.py || exit 1
