#!/bin/bash
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
(rocm-smi --showuniqueid > gpurun_out/smi.log 2>&1 || true); grep -i "unique id" gpurun_out/smi.log | tail -1
TESTS="tests/test_gpu_parity.py tests/test_gpu_log.py" bash scripts/gpu_tests.sh || exit $?
SWEEP_NAMES=${SWEEP_NAMES:-grw0,grw1,r0,r13,r1028,r1284} \
  timeout -k 10 300 python scripts/sweep_unpack.py > gpurun_out/sweep7.log 2>&1 || { echo "sweep failed"; tail -5 gpurun_out/sweep7.log; exit 4; }
tail -1 gpurun_out/sweep7.log
