#!/bin/bash
# Round 4: the default bench line, its rocprofv3 kernel stats, and the config-4 traffic counters.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py > gpurun_out/bench.log 2>&1 || { tail -5 gpurun_out/bench.log; exit 1; }
tail -c 2500 gpurun_out/bench.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/benchprof -o bench -- python3 -u bench.py --steps 20 --warmup 5 > gpurun_out/benchprof.log 2>&1 || exit $?
bash scripts/pmc_c4.sh > gpurun_out/pmc_c4.log 2>&1; tail -3 gpurun_out/pmc_c4.log
