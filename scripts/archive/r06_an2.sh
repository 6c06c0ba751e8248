#!/bin/bash
# round 6: analytics parity + the long-record unpack parity, config-4 A/B, config-5 unpack timing
set -u
export TMPDIR=/tmp
OUT=gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_analytics.py tests/test_gpu_unpack_long.py tests/test_gpu_scan.py \
  > $OUT/r06_an2_tests.log 2>&1 || { tail -40 $OUT/r06_an2_tests.log; exit 1; }
tail -3 $OUT/r06_an2_tests.log
timeout -k 10 600 bash scripts/ab_c4.sh || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c4r6b -o c4 -- \
  python3 scripts/c4_only.py > $OUT/c4r6b.log 2>&1 || { tail -20 $OUT/c4r6b.log; exit 1; }
python3 scripts/kstats.py $OUT/c4r6b 14 || true
python3 scripts/c4_dispatch.py $(ls $OUT/c4r6b/*kernel_trace.csv $OUT/c4r6b/*/*kernel_trace.csv 2>/dev/null | head -1) || true
timeout -k 10 300 python3 scripts/c5_only.py > $OUT/c5r6.log 2>&1 || { tail -20 $OUT/c5r6.log; exit 1; }
tail -2 $OUT/c5r6.log
