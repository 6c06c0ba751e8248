#!/bin/bash
# pack ablations on config 3 (diag build): 0 product, 1 = no unit stores, 2 = no CRC work
set -u
mkdir -p gpurun_out
: > gpurun_out/c3pabl.log
for v in 1 2; do
  timeout -k 10 200 python -u scripts/c3_probe.py ${CASES:-mixed,uniform_768} 3 $v >> gpurun_out/c3pabl.log 2>&1 || exit $?
done
grep -v amdgpu.ids gpurun_out/c3pabl.log
