#!/bin/bash
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
(rocm-smi --showuniqueid > gpurun_out/smi.log 2>&1 || true); grep -i "unique id" gpurun_out/smi.log | tail -1
TESTS="tests/test_gpu_flowtab.py tests/test_gpu_analytics.py tests/test_gpu_comm.py tests/test_compat_gpu.py" bash scripts/gpu_tests.sh || exit $?
SWEEP_NAMES=${SWEEP_NAMES:-grw0,grw1,grw4112,grw4116,grw4117,grw4096,grw4100,r0,r1028,r1284} \
  timeout -k 10 300 python scripts/sweep_unpack.py > gpurun_out/sweep6.log 2>&1 || { echo "sweep failed"; tail -5 gpurun_out/sweep6.log; exit 4; }
tail -1 gpurun_out/sweep6.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/scanprof -o scan -- python3 scripts/scan_profile.py > gpurun_out/scanprof.log 2>&1
echo "scanprof rc=$?"; tail -2 gpurun_out/scanprof.log
