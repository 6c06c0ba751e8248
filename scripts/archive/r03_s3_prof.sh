#!/bin/bash
# Round 3, session 3 profiles: headline + whole-bench kernel stats and HBM counters
# (r03_final_prof.sh), then the config-4 and config-5 kernel traces (csv).
set -u
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
bash scripts/archive/r03_final_prof.sh || exit $?
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c4csv -o c4 \
    -- python3 -u scripts/c4_only.py > $OUT/c4csv.log 2>&1 || exit $?
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c5csv -o c5 \
    -- python3 -u scripts/scan_time.py > $OUT/c5csv.log 2>&1 || exit $?
tail -3 $OUT/c5csv.log
