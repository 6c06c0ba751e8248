#!/bin/bash
# Round 5: the column scan fused (hist adds chunk partials + flow totals, one scan kernel):
# analytics parity, config-4 timing, a kernel trace of it.
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
step an_tests 600 python -u -m pytest tests/test_gpu_analytics.py tests/test_gpu_report.py tests/test_gpu_pcap.py tests/test_gpu_comm.py -m gpu -x -q --timeout 120 --timeout-method thread
step c4 300 python -u scripts/c4_only.py
rm -rf gpurun_out/c4prof
step c4prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c4prof -o c4 -- python3 -u scripts/c4_only.py
python3 scripts/kstats.py gpurun_out/c4prof 16
