#!/bin/bash
# Round 5: the chain hypothesis without link / block-count scan (scan_chain_*): scan parity
# tests, the config-5 scan timing, and a kernel trace of it.
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
step scan_tests 600 python -u -m pytest tests/test_gpu_scan.py tests/test_gpu_tcp_tx.py -m gpu -x -q --timeout 120 --timeout-method thread
step scan_time 120 python -u scripts/scan_time.py
rm -rf gpurun_out/scanprof
step scanprof 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/scanprof -o sc -- python -u scripts/scan_time.py
python3 scripts/scan_trace.py gpurun_out/scanprof
