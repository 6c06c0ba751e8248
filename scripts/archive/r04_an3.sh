#!/bin/bash
# Round 4: analytics tests, config-4 timing + kernel trace, SQ counters of the update kernel.
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
step an_tests 600 python -u -m pytest tests/test_gpu_analytics.py tests/test_gpu_report.py tests/test_gpu_pcap.py -m gpu -x -q --timeout 120 --timeout-method thread
step c4 180 python -u scripts/c4_only.py
step c4prof 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c4prof3 -o c4 -- python3 -u scripts/c4_only.py
python3 scripts/c4_dispatch.py gpurun_out/c4prof3/c4_kernel_trace.csv
step c4sq 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY --kernel-trace --output-format csv -d gpurun_out/c4sq -o sq -- python3 -u scripts/c4_only.py
python3 scripts/sq_update.py gpurun_out/c4sq
