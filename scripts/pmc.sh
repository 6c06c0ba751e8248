#!/bin/bash
# HBM traffic counters for the bench kernels: one rocprofv3 pass per counter group
# (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass), kernel-trace only, no sys/runtime
# trace.  Output: gpurun_out/pmc_{fetch,write}/...
set -u
export TMPDIR=/tmp
OUT=gpurun_out
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv \
      -d $OUT/pmc_$c -o pmc -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline \
      > $OUT/pmc_$c.log 2>&1
  rc=$?
  echo "pmc $c rc=$rc"; tail -n 3 $OUT/pmc_$c.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
python scripts/parse_pmc.py $OUT
