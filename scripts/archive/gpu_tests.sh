#!/bin/bash
# GPU tests (all, or the files given), then optional extra steps.  A fault / abort / timeout
# ends the script before anything else touches the GPU.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
(rocm-smi --showserial --showuniqueid --showclocks > gpurun_out/smi.log 2>&1 || true)
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -q --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pt.log 2>&1
rc=$?
tail -40 gpurun_out/pt.log
if [ $rc -ge 124 ] || grep -q -i "memory access fault\|core dumped\|illegal" gpurun_out/pt.log; then
  echo "FATAL: GPU error in tests (rc=$rc) -- stopping"; exit 3
fi
if [ -n "${SWEEP_NAMES:-}" ]; then
  timeout -k 10 300 python scripts/sweep_unpack.py > gpurun_out/sweep.log 2>&1
  echo "sweep rc=$?"; tail -1 gpurun_out/sweep.log
fi
exit $rc
