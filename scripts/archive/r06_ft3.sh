#!/bin/bash
# round 6: FindFlow small-table path (two workgroups per CU) + TCP walk interleave -- parity, A/B, sweep
set -u
export TMPDIR=/tmp
OUT=gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_flowtab.py tests/test_gpu_tcp_tx.py tests/test_gpu_scan.py \
  > $OUT/r06_ft3_tests.log 2>&1 || { tail -40 $OUT/r06_ft3_tests.log; exit 1; }
tail -3 $OUT/r06_ft3_tests.log
timeout -k 10 300 python3 scripts/ft_time.py || exit 1
MGENX_LIB_OVERRIDE=$PWD/mgen_amd/libmgenx_ab.so timeout -k 10 300 python3 scripts/ft_time.py || exit 1
D=$PWD/mgen_amd/libmgenx_diag.so
for g in 1 2 4 8; do
  MGENX_FT_GMUL=$g MGENX_LIB_OVERRIDE=$D timeout -k 10 300 python3 scripts/ft_time.py || exit 1
  MGENX_FT_MODE=1 MGENX_FT_GMUL=$g MGENX_LIB_OVERRIDE=$D timeout -k 10 300 python3 scripts/ft_time.py || exit 1
done
MGENX_FT_KCAP=0 MGENX_LIB_OVERRIDE=$D timeout -k 10 300 python3 scripts/ft_time.py || exit 1
timeout -k 10 600 bash scripts/ab_tcp.sh || exit 1
