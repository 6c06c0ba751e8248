#!/bin/bash
# Round 5: worker CRC through LDS shift tables, no blanket acquire -- tests, latency, stamps.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  tail -${TAILN:-4} "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "STEP $name FAILED rc=$rc"; exit $rc; fi
}
step wk_tests 600 python -u -m pytest tests/test_gpu_worker.py tests/test_compat_gpu.py tests/test_gpu_pack_msgs.py -m gpu -x -q --timeout 120 --timeout-method thread
step shim_lat 120 ./tests/cpp/shim_latency 2000
step wk_stamps 200 python -u scripts/wk_stamps.py
