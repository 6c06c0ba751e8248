#!/bin/bash
# Round 4: TCP transmit (one sync per call) -- parity tests and config-5 timing.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_tcp_tx.py tests/test_gpu_scan.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tcp_tests.log 2>&1; rc=$?
tail -3 gpurun_out/tcp_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/c5_only.py > gpurun_out/c5.log 2>&1 || exit $?
tail -c 800 gpurun_out/c5.log
