#!/bin/bash
# Round 4: persistent order kernel -- analytics parity, config-4 timing, kernel trace.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  tail -${TAILN:-12} "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "STEP $name FAILED rc=$rc"; exit $rc; fi
}
step an_tests 600 python -u -m pytest tests/test_gpu_analytics.py tests/test_gpu_report.py -m gpu -x -q --timeout 120 --timeout-method thread
step an_order 300 python -u scripts/an_order.py
step upd_prof 200 python3 -u scripts/upd_prof.py
step c4prof 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c4prof4 -o c4 -- python3 -u scripts/c4_only.py
python3 scripts/c4_dispatch.py gpurun_out/c4prof4/c4_kernel_trace.csv
