#!/bin/bash
# Round 4: analytics / FindFlow / pcap2mgen tests, config-4 timing and kernel trace.
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
step an_tests 600 python -u -m pytest tests/test_gpu_worker.py tests/test_gpu_pack_msgs.py tests/test_gpu_analytics.py tests/test_gpu_flowtab.py tests/test_gpu_pcap.py tests/test_gpu_report.py tests/test_gpu_comm.py -m gpu -x -v --timeout 120 --timeout-method thread
step c4 180 python -u scripts/c4_only.py
step c4prof 240 rocprofv3 --kernel-trace --stats -d gpurun_out/c4prof -o c4 -- python3 -u scripts/c4_only.py
find gpurun_out/c4prof -name '*kernel_stats.csv' -exec cp {} gpurun_out/c4_kernel_stats.csv \;
python3 scripts/kstats.py gpurun_out/c4prof 20
TAILN=25 step var 300 env VARIANTS=${VARIANTS:-0,33,20} python -u scripts/var_shapes.py
step mailbox 60 ./scripts/diag/mailbox_probe 3000
step scan_full 400 python -u -m pytest tests/test_gpu_scan.py -m gpu -x -v -k full_size --timeout 300 --timeout-method thread
step compat 300 python -u -m pytest tests/test_compat_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread
step shim_lat 120 ./tests/cpp/shim_latency 2000
cp gpurun_out/shim_lat.log gpurun_out/shim_latency.json
