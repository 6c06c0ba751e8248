#!/bin/bash
# Config-4 HBM traffic: one rocprofv3 pass per counter, kernel-trace only, then a plain
# kernel-trace pass for the durations; parse into profiles/r04/traffic_config4.json.
set -u
export TMPDIR=/tmp
OUT=gpurun_out
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv \
      -d $OUT/pmc4_$c -o pmc -- python3 scripts/traffic_c4.py > $OUT/pmc4_$c.log 2>&1
  rc=$?
  echo "pmc $c rc=$rc"; tail -n 2 $OUT/pmc4_$c.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $OUT/pmc4_time -o t -- python3 scripts/traffic_c4.py > $OUT/pmc4_time.log 2>&1 || exit $?
python3 scripts/parse_pmc_c4.py $OUT
