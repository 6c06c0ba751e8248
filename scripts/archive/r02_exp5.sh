#!/bin/bash
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
(rocm-smi --showuniqueid > gpurun_out/smi.log 2>&1 || true); grep -i unique gpurun_out/smi.log | tail -1
SWEEP_NAMES=${SWEEP_NAMES:-grw0,grw1,grw4112,grw4116,grw4117,grw4096,grw4100,r0,r1028,r1284} \
  timeout -k 10 300 python scripts/sweep_unpack.py > gpurun_out/sweep5.log 2>&1 || { echo "sweep failed"; tail -5 gpurun_out/sweep5.log; exit 4; }
tail -1 gpurun_out/sweep5.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/scanprof -o scan -- python3 scripts/scan_profile.py > gpurun_out/scanprof.log 2>&1
echo "scanprof rc=$?"; tail -2 gpurun_out/scanprof.log
find gpurun_out/scanprof -name "*stats*"
