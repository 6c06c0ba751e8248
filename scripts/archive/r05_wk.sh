#!/bin/bash
# Round 5: the resident worker v2 (device-memory request block, Unpack + CRC in one reply,
# MgenAnalytic::Update) -- its tests, the shim tests, the shim latency program.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  tail -${TAILN:-8} "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "STEP $name FAILED rc=$rc"; exit $rc; fi
}
step wk_tests 600 python -u -m pytest tests/test_gpu_worker.py tests/test_compat_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread
step shim_lat 120 ./tests/cpp/shim_latency 2000
MGENX_WORKER_HOST_MAILBOX=1 step shim_lat_host 120 ./tests/cpp/shim_latency 2000
step an_tests 600 python -u -m pytest tests/test_gpu_analytics.py -m gpu -x -q --timeout 120 --timeout-method thread
