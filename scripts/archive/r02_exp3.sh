#!/bin/bash
set -u
mkdir -p gpurun_out
TESTS="tests/test_compat_gpu.py tests/test_gpu_pack_msgs.py tests/test_gpu_comm.py" bash scripts/gpu_tests.sh || exit $?
timeout -k 10 120 python scripts/probe_write_after_read.py > gpurun_out/war.log 2>&1; echo "war rc=$?"; tail -2 gpurun_out/war.log
