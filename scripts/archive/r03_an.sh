#!/bin/bash
# analytics: parity tests, then config 4 timing and its kernel trace
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_analytics.py tests/test_gpu_flowtab.py tests/test_gpu_report.py tests/test_gpu_pcap.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/an_tests.log 2>&1
rc=$?; tail -3 gpurun_out/an_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/c4_only.py > gpurun_out/c4.log 2>&1 || exit 1
tail -1 gpurun_out/c4.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c4prof -o c4 -- python -u scripts/c4_only.py > gpurun_out/c4prof.log 2>&1 || exit 1
find gpurun_out/c4prof -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'head -12 {}'
timeout -k 10 300 python -u scripts/an_abl.py > gpurun_out/an_abl.log 2>&1; cat gpurun_out/an_abl.log
