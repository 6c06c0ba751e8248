#!/bin/bash
# scan tests (pruning + marked chain), config-5 timing and kernel trace
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  tail -${TAILN:-15} "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "STEP $name FAILED rc=$rc"; exit $rc; fi
}
step scan_tests 400 python -u -m pytest tests/test_gpu_scan.py tests/test_gpu_shard_cpp.py -m gpu -x -q --timeout 200 --timeout-method thread
step c5 120 python -u scripts/c5_only.py
step scan_time 120 python -u scripts/scan_time.py
step c5prof 180 rocprofv3 --kernel-trace --stats -d gpurun_out/c5prof -o c5 -- python3 -u scripts/scan_time.py
