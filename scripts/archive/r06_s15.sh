#!/bin/bash
# round 6: header-only decode with headers in flight -- parity, timing, A/B
set -u
export TMPDIR=/tmp
OUT=gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_flowtab.py tests/test_gpu_parity.py tests/test_gpu_unpack_var.py tests/test_gpu_pcap.py tests/test_gpu_binlog.py \
  tests/test_gpu_scan.py tests/test_gpu_tcp_rx.py tests/test_gpu_analytics.py \
  > $OUT/r06_s15_tests.log 2>&1 || { tail -40 $OUT/r06_s15_tests.log; exit 1; }
tail -3 $OUT/r06_s15_tests.log
timeout -k 10 300 python3 -u scripts/hdr_time.py || exit 1
timeout -k 10 300 python3 -u scripts/hdr_time.py || exit 1
timeout -k 10 300 python3 -u scripts/ft_time.py || exit 1
