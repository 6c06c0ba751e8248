#!/bin/bash
# rocprofv3 kernel-trace + stats of the bench (headline only), then the PMC traffic passes.
set -u
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run \
    -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras > $OUT/prof_bench.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -n 1 $OUT/prof_bench.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash scripts/pmc.sh
