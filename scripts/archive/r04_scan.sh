#!/bin/bash
# Round 4: scan parity after the two-pass offsets scan, then its timing (one-workgroup form via
# the diagnostics switch for comparison).
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
step scan_tests 600 python -u -m pytest tests/test_gpu_scan.py tests/test_gpu_shard_cpp.py tests/test_gpu_tcp_rx.py -m gpu -x -q --timeout 120 --timeout-method thread
step scan_time 200 python -u scripts/scan_time.py
DIAG=1 MGENX_SCAN_OFF1=1 step scan_time_off1 200 python -u scripts/scan_time.py
DIAG=1 step scan_time_diag 200 python -u scripts/scan_time.py
