#!/bin/bash
# config-3 HBM traffic: one rocprofv3 pass per counter, kernel-trace only; then the kernel
# trace + stats of the same probe for the durations
set -u
export TMPDIR=/tmp
OUT=gpurun_out
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv \
      -d $OUT/pmc_$c -o pmc -- python3 scripts/traffic_c3.py > $OUT/pmc_$c.log 2>&1
  rc=$?
  echo "pmc $c rc=$rc"; tail -n 2 $OUT/pmc_$c.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c3trace -o c3 \
    -- python3 scripts/traffic_c3.py > $OUT/c3trace.log 2>&1 || exit $?
python3 scripts/parse_pmc_c3.py $OUT
