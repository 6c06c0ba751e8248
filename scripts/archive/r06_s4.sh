#!/bin/bash
# round 6: skeleton with chunk summaries + var-kernel record order: parity, A/B, profiles
set -u
export TMPDIR=/tmp
OUT=gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_analytics.py tests/test_gpu_unpack_var.py tests/test_gpu_parity.py \
  tests/test_gpu_unpack_long.py > $OUT/r06_s4_tests.log 2>&1 || { tail -40 $OUT/r06_s4_tests.log; exit 1; }
tail -3 $OUT/r06_s4_tests.log
timeout -k 10 600 bash scripts/ab_c4.sh || exit 1
timeout -k 10 300 python3 scripts/skel_prof.py || exit 1
for k in 1 2; do
  timeout -k 10 300 python3 scripts/c3_only.py 2 | tail -1 || exit 1
  MGENX_LIB_OVERRIDE=$PWD/mgen_amd/libmgenx_ab.so timeout -k 10 300 python3 scripts/c3_only.py 2 | tail -1 || exit 1
done
