#!/bin/bash
# Round 5: the workgroup-per-flow update (flow_update_wg_kernel) -- analytics parity, then
# config-4 timing with it and with the wave kernel (MGENX_FLOW_UPDATE=wave).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  tail -${TAILN:-6} "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "STEP $name FAILED rc=$rc"; exit $rc; fi
}
step an_tests 600 python -u -m pytest tests/test_gpu_analytics.py tests/test_gpu_report.py tests/test_gpu_worker.py -m gpu -x -q --timeout 120 --timeout-method thread
step c4_wg 300 python -u scripts/c4_only.py
MGENX_FLOW_UPDATE=wave step c4_wave 300 python -u scripts/c4_only.py
