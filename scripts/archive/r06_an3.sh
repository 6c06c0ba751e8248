#!/bin/bash
# round 6: analytics parity, config-4 A/B, skeleton phase cycles, kernel trace
set -u
export TMPDIR=/tmp
OUT=gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_analytics.py tests/test_gpu_worker.py \
  > $OUT/r06_an3_tests.log 2>&1 || { tail -40 $OUT/r06_an3_tests.log; exit 1; }
tail -3 $OUT/r06_an3_tests.log
timeout -k 10 600 bash scripts/ab_c4.sh || exit 1
timeout -k 10 300 python3 scripts/skel_prof.py || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c4r6c -o c4 -- \
  python3 scripts/c4_only.py > $OUT/c4r6c.log 2>&1 || { tail -20 $OUT/c4r6c.log; exit 1; }
python3 scripts/c4_dispatch.py $(ls $OUT/c4r6c/*kernel_trace.csv $OUT/c4r6c/*/*kernel_trace.csv 2>/dev/null | head -1) || true
