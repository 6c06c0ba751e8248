#!/bin/bash
# Round 3 profiles: rocprofv3 kernel-trace + stats of the whole bench (extras on, no CPU
# baseline), then the FETCH_SIZE / WRITE_SIZE passes (scripts/pmc.sh) -> traffic_r03.json.
set -u
export TMPDIR=/tmp ROUND=r03
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run \
    -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/prof_bench.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -c 600 $OUT/prof_bench.log
if [ $rc -ne 0 ]; then exit $rc; fi
if [ "${PMC:-1}" = "1" ]; then bash scripts/pmc.sh; fi
