#!/bin/bash
# round 6: A/B (HEAD build in libmgenx_ab.so) of the header-only ring and FindFlow's first call
set -u
export TMPDIR=/tmp
OUT=gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_flowtab.py tests/test_gpu_pcap.py > $OUT/r06_s16_tests.log 2>&1 || { tail -40 $OUT/r06_s16_tests.log; exit 1; }
tail -3 $OUT/r06_s16_tests.log
for k in 1 2; do
  echo new; timeout -k 10 300 python3 -u scripts/hdr_time.py || exit 1
  echo old; MGENX_LIB_OVERRIDE=$PWD/mgen_amd/libmgenx_ab.so timeout -k 10 300 python3 -u scripts/hdr_time.py || exit 1
done
echo new; timeout -k 10 300 python3 -u scripts/ft_time.py || exit 1
echo old; MGENX_LIB_OVERRIDE=$PWD/mgen_amd/libmgenx_ab.so timeout -k 10 300 python3 -u scripts/ft_time.py || exit 1
