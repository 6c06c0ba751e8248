#!/bin/bash
# round 6: window-parallel MgenAnalytic::Update -- analytics parity, then config-4 A/B against
# the round-5 library (mgen_amd/libmgenx_ab.so) and a kernel trace of config 4
set -u
export TMPDIR=/tmp
OUT=gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_analytics.py tests/test_gpu_worker.py tests/test_gpu_comm.py \
  > $OUT/r06_an_tests.log 2>&1 || { tail -40 $OUT/r06_an_tests.log; exit 1; }
tail -3 $OUT/r06_an_tests.log
timeout -k 10 600 bash scripts/ab_c4.sh || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c4r6 -o c4 -- \
  python3 scripts/c4_only.py > $OUT/c4r6.log 2>&1 || { tail -20 $OUT/c4r6.log; exit 1; }
python3 scripts/kstats.py $OUT/c4r6 24 || true
python3 scripts/c4_dispatch.py $(ls $OUT/c4r6/*kernel_trace.csv $OUT/c4r6/*/*kernel_trace.csv 2>/dev/null | head -1) || true
