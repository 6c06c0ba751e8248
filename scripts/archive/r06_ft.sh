#!/bin/bash
# round 6: FindFlow -- parity, then new vs round-5 library and the insert kernel's ablations
set -u
export TMPDIR=/tmp
OUT=gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_flowtab.py > $OUT/r06_ft_tests.log 2>&1 || { tail -40 $OUT/r06_ft_tests.log; exit 1; }
tail -3 $OUT/r06_ft_tests.log
for k in 1 2; do
  timeout -k 10 300 python3 scripts/ft_time.py || exit 1
  MGENX_LIB_OVERRIDE=$PWD/mgen_amd/libmgenx_ab.so timeout -k 10 300 python3 scripts/ft_time.py || exit 1
done
for m in 0 1 2; do
  MGENX_FT_MODE=$m MGENX_LIB_OVERRIDE=$PWD/mgen_amd/libmgenx_diag.so timeout -k 10 300 python3 scripts/ft_time.py || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ftr6 -o ft -- \
  python3 scripts/ft_time.py > $OUT/ftr6.log 2>&1 || { tail -20 $OUT/ftr6.log; exit 1; }
python3 scripts/kstats.py $OUT/ftr6 14 || true
