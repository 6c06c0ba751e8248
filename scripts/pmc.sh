#!/bin/bash
# HBM traffic counters: one rocprofv3 pass per counter (FETCH_SIZE and WRITE_SIZE do not
# fit one TCC pass), kernel-trace only (no sys/runtime trace), over scripts/traffic_probe.py.
set -u
export TMPDIR=/tmp
OUT=gpurun_out
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv \
      -d $OUT/pmc_$c -o pmc -- python3 scripts/traffic_probe.py > $OUT/pmc_$c.log 2>&1
  rc=$?
  echo "pmc $c rc=$rc"; tail -n 2 $OUT/pmc_$c.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
python3 scripts/parse_pmc.py $OUT
