#!/bin/bash
# FindFlow tests + config-4 timing + kernel trace
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
step ft_tests 400 python -u -m pytest tests/test_gpu_flowtab.py tests/test_gpu_analytics.py tests/test_gpu_pcap.py tests/test_compat_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread
step c4 120 python -u scripts/c4_only.py
step c4csv 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c4csv2 -o c4 -- python3 -u scripts/c4_only.py
