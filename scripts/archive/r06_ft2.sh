#!/bin/bash
# round 6: FindFlow small-table path + TCP walk zero passes -- parity, then A/B
set -u
export TMPDIR=/tmp
OUT=gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_flowtab.py tests/test_gpu_tcp_tx.py tests/test_gpu_scan.py tests/test_gpu_analytics.py \
  > $OUT/r06_ft2_tests.log 2>&1 || { tail -40 $OUT/r06_ft2_tests.log; exit 1; }
tail -3 $OUT/r06_ft2_tests.log
for k in 1 2; do
  timeout -k 10 300 python3 scripts/ft_time.py || exit 1
  MGENX_LIB_OVERRIDE=$PWD/mgen_amd/libmgenx_ab.so timeout -k 10 300 python3 scripts/ft_time.py || exit 1
done
MGENX_FT_MODE=1 MGENX_LIB_OVERRIDE=$PWD/mgen_amd/libmgenx_diag.so timeout -k 10 300 python3 scripts/ft_time.py || exit 1
timeout -k 10 600 bash scripts/ab_tcp.sh || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ftr6b -o ft -- \
  python3 scripts/ft_time.py > $OUT/ftr6b.log 2>&1 || { tail -20 $OUT/ftr6b.log; exit 1; }
python3 scripts/kstats.py $OUT/ftr6b 10 || true
