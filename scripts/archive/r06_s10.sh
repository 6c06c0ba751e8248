#!/bin/bash
# round 6: mgenx_flow_span (pcap2mgen's slot sizing on the device) -- parity, pcap timing
set -u
export TMPDIR=/tmp
OUT=gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_flowtab.py tests/test_gpu_pcap.py tests/test_golden_cpu.py > $OUT/r06_s10_tests.log 2>&1 || { tail -40 $OUT/r06_s10_tests.log; exit 1; }
tail -3 $OUT/r06_s10_tests.log
timeout -k 10 300 python3 scripts/pcap_time.py || exit 1
MGENX_LIB_OVERRIDE=$PWD/mgen_amd/libmgenx_ab.so timeout -k 10 300 python3 scripts/pcap_time.py || true
