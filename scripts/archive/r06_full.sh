#!/bin/bash
# Round 6: the whole -m gpu suite, the default bench line, and the headline-only kernel stats
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/suite_r06.log 2>&1; rc=$?
tail -4 gpurun_out/suite_r06.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u bench.py > gpurun_out/bench_r06.log 2>&1 || { tail -5 gpurun_out/bench_r06.log; exit 1; }
tail -c 3000 gpurun_out/bench_r06.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/benchprof_r06 -o bench -- python3 -u bench.py --no-extras --steps 50 --warmup 5 > gpurun_out/benchprof_r06.log 2>&1 || exit $?
python3 scripts/kstats.py gpurun_out/benchprof_r06 6 || true
