#!/bin/bash
# all GPU tests + bench (with extras, no CPU baseline) + scan profile
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_tests.sh || exit $?
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_b.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/bench_b.log; exit 5; }
bash scripts/r02_scan.sh
