#!/bin/bash
# Round-2 measurement call: every GPU test, the bench (headline + extras + CPU baseline),
# a rocprofv3 kernel trace of the bench, and the FETCH/WRITE counter passes.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
(rocm-smi --showuniqueid > gpurun_out/smi.log 2>&1 || true); grep -i "unique id" gpurun_out/smi.log | tail -1
bash scripts/gpu_tests.sh || exit $?
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_full.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/bench_full.log; exit 5; }
tail -c 300 gpurun_out/bench_full.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash scripts/pmc.sh
