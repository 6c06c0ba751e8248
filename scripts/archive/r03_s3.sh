#!/bin/bash
# Round 3, session 3: analytics tests + config-4 timing + kernel trace, then the var-kernel shapes.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  tail -${TAILN:-15} "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "STEP $name FAILED rc=$rc"; exit $rc; fi
}
step an_tests 300 python -u -m pytest tests/test_gpu_analytics.py tests/test_gpu_report.py tests/test_gpu_comm.py -m gpu -x -q --timeout 120 --timeout-method thread
step c4 120 python -u scripts/c4_only.py
step c4prof 180 rocprofv3 --kernel-trace --stats -d gpurun_out/c4prof -o c4 -- python3 -u scripts/c4_only.py
find gpurun_out/c4prof -name '*kernel_stats.csv' -exec cp {} gpurun_out/c4_kernel_stats.csv \;
TAILN=25 step var 300 env VARIANTS=${VARIANTS:-0,20,24,30,31,32,33,22} python -u scripts/var_shapes.py
