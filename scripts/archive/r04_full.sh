#!/bin/bash
# Round 4: the whole -m gpu suite, the default bench line, its rocprofv3 kernel stats, and the
# config-4 traffic counters.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/suite.log 2>&1; rc=$?
tail -4 gpurun_out/suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/bench.log 2>&1 || { tail -5 gpurun_out/bench.log; exit 1; }
tail -c 1500 gpurun_out/bench.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/benchprof -o bench -- python3 -u bench.py --steps 20 --warmup 5 > gpurun_out/benchprof.log 2>&1 || exit $?
bash scripts/pmc_c4.sh > gpurun_out/pmc_c4.log 2>&1; tail -3 gpurun_out/pmc_c4.log
