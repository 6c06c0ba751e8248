#!/bin/bash
# round 6 session start: the changed tests (TCP doc pin, worker / shim after the quiesce fix),
# then the headline's HBM counter passes -> profiles/traffic_r06.json
set -u
export TMPDIR=/tmp
OUT=gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_tcp_tx.py tests/test_gpu_worker.py tests/test_compat_gpu.py tests/test_oracle_pins.py \
  > $OUT/r06_base_tests.log 2>&1 || { tail -30 $OUT/r06_base_tests.log; exit 1; }
tail -3 $OUT/r06_base_tests.log
ROUND=r06 bash scripts/pmc.sh
