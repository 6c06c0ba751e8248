#!/bin/bash
# Round 5: small order tiles for small calls -- analytics parity and config-4 timing + trace.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  tail -${TAILN:-3} "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "STEP $name FAILED rc=$rc"; exit $rc; fi
}
step an_tests 600 python -u -m pytest tests/test_gpu_analytics.py tests/test_gpu_report.py tests/test_gpu_pcap.py -m gpu -x -q --timeout 120 --timeout-method thread
step c4prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c4prof5 -o c4 -- python3 -u scripts/c4_only.py
python3 scripts/c4_dispatch.py gpurun_out/c4prof5/c4_kernel_trace.csv
