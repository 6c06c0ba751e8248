#!/bin/bash
# Round 2, first call: GPU tests, the bench, then the store-placement ablation sweep of the
# headline kernel and the memory-pattern probes.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt.log 2>&1
rc=$?
tail -3 gpurun_out/pt.log
if [ $rc -ge 124 ] || grep -q -i "illegal memory\|memory access fault\|core dumped" gpurun_out/pt.log; then
  echo "FATAL: GPU error in tests (rc=$rc) -- stopping"; exit 3
fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/bench.log; exit 4; }
tail -c 600 gpurun_out/bench.log
SWEEP_NAMES=r0,r1040,r1088,r1152,r1168,r1028,r1284,r1796,r1026,r1032,grw0,grw1,grw3,grw4,read_8192,fill_rows \
  timeout -k 10 300 python scripts/sweep_unpack.py > gpurun_out/sweep.log 2>&1
echo "sweep rc=$?"; tail -1 gpurun_out/sweep.log
