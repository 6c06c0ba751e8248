#!/bin/bash
# GPU tests then the unpack ablation sweep.  Any HIP/GPU error, fault, abort or timeout in
# the tests ends the script before anything else touches the GPU.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q ${PYTEST_ARGS:-} > gpurun_out/pt.log 2>&1
rc=$?
tail -3 gpurun_out/pt.log
if [ $rc -ge 124 ] || grep -q -i "illegal memory\|HIP error\|hipError\|memory access fault\|core dumped" gpurun_out/pt.log; then
  echo "FATAL: GPU error in tests (rc=$rc) -- stopping"; exit 3
fi
if [ "${SWEEP:-1}" = "1" ]; then
  timeout -k 10 300 python scripts/sweep_unpack.py > gpurun_out/sweep.log 2>&1
  echo "sweep rc=$?"; tail -1 gpurun_out/sweep.log
fi
