#!/bin/bash
# round 6: FindFlow small-table path without the ticket fence -- parity, A/B, grid sweep
set -u
export TMPDIR=/tmp
OUT=gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_flowtab.py > $OUT/r06_ft4_tests.log 2>&1 || { tail -40 $OUT/r06_ft4_tests.log; exit 1; }
tail -3 $OUT/r06_ft4_tests.log
timeout -k 10 300 python3 scripts/ft_time.py || exit 1
MGENX_LIB_OVERRIDE=$PWD/mgen_amd/libmgenx_ab.so timeout -k 10 300 python3 scripts/ft_time.py || exit 1
D=$PWD/mgen_amd/libmgenx_diag.so
for g in 1 2 4; do
  MGENX_FT_GMUL=$g MGENX_LIB_OVERRIDE=$D timeout -k 10 300 python3 scripts/ft_time.py || exit 1
  MGENX_FT_MODE=1 MGENX_FT_GMUL=$g MGENX_LIB_OVERRIDE=$D timeout -k 10 300 python3 scripts/ft_time.py || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ftr6c -o ft -- \
  python3 scripts/ft_time.py > $OUT/ftr6c.log 2>&1 || { tail -20 $OUT/ftr6c.log; exit 1; }
python3 scripts/kstats.py $OUT/ftr6c 8 || true
