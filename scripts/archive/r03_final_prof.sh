#!/bin/bash
# Round 3 profiles (everything lands in gpurun_out/, merged back by gpurun):
#   1. rocprofv3 --kernel-trace --stats of the headline alone (bench.py --no-extras)
#   2. the same over the whole bench (extras on) + the FETCH_SIZE / WRITE_SIZE passes of
#      scripts/pmc.sh -> traffic_r03.json (scripts/archive/r03_prof.sh)
#   3. the config-3 counter passes and flushed kernel trace (scripts/pmc_c3.sh)
set -u
export ROUND=r03 TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_head -o head \
    -- python3 bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-extras > $OUT/prof_head.log 2>&1
rc=$?; echo "headline rocprof rc=$rc"; tail -c 400 $OUT/prof_head.log
[ $rc -ne 0 ] && exit $rc
bash scripts/archive/r03_prof.sh || exit $?
rm -rf $OUT/pmc_FETCH_SIZE $OUT/pmc_WRITE_SIZE
bash scripts/pmc_c3.sh || exit $?
cp profiles/r03/traffic_config3.json $OUT/traffic_config3_r03.json
