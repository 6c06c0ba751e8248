#!/bin/bash
# Round 4: worker + analytics tests, config-4 timing and kernel trace (csv), shim latency.
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
step an_tests 600 python -u -m pytest tests/test_gpu_worker.py tests/test_gpu_pack_msgs.py tests/test_gpu_analytics.py tests/test_gpu_flowtab.py tests/test_gpu_report.py tests/test_gpu_comm.py tests/test_gpu_pcap.py -m gpu -x -q --timeout 120 --timeout-method thread
step c4 180 python -u scripts/c4_only.py
step c4prof 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c4prof2 -o c4 -- python3 -u scripts/c4_only.py
python3 scripts/kstats.py gpurun_out/c4prof2 24
step compat 300 python -u -m pytest tests/test_compat_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread
step shim_lat 120 ./tests/cpp/shim_latency 2000
