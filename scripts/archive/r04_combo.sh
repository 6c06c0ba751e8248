#!/bin/bash
# Round 4: worker checks + shim latency, analytics parity (product + diagnostics workgroup
# path), config-4 timing.
set -u
bash scripts/archive/r04_wk.sh || exit $?
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_analytics.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/an_tests.log 2>&1; rc=$?
tail -3 gpurun_out/an_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -u scripts/c4_only.py > gpurun_out/c4.log 2>&1 || exit $?
cut -c1-600 gpurun_out/c4.log | tail -2
