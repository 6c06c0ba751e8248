#!/bin/bash
# round 6: segmented Update (close chain + speculative segment starts + verify) -- parity, A/B
set -u
export TMPDIR=/tmp
OUT=gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_analytics.py tests/test_gpu_pcap.py tests/test_gpu_report.py > $OUT/r06_s17_tests.log 2>&1 || { tail -40 $OUT/r06_s17_tests.log; exit 1; }
tail -3 $OUT/r06_s17_tests.log
for k in 1 2; do
  for sg in 1 0; do
    MGENX_FLOW_SEGMENTS=$sg timeout -k 10 200 python -u scripts/c4_only.py 2>/dev/null | python3 -c "
import json,sys
d=json.loads(sys.stdin.read().strip().splitlines()[-1])
r=d.get('rank_share_at_8') or {}
print('seg=$sg', d['reduce_ms'], r.get('reduce_ms'), d['rows_pipeline']['reduce_ms'])" || exit 1
  done
done
MGENX_FLOW_SEGMENTS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/segprof -o seg -- \
  python3 scripts/c4_only.py > $OUT/segprof.log 2>&1 || { tail -20 $OUT/segprof.log; exit 1; }
python3 scripts/kstats.py $OUT/segprof 12 || true
