#!/bin/bash
# Round 6 end: smoke(), the whole -m gpu suite and the default bench line on the final tree
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r06z.log 2>&1 || { tail -5 gpurun_out/smoke_r06z.log; exit 1; }
tail -1 gpurun_out/smoke_r06z.log
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/suite_r06z.log 2>&1; rc=$?
tail -2 gpurun_out/suite_r06z.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u bench.py > gpurun_out/bench_r06z.log 2>&1 || { tail -5 gpurun_out/bench_r06z.log; exit 1; }
tail -c 300 gpurun_out/bench_r06z.log
