#!/bin/bash
# config-3 probe: the product kernels, then the unsorted general unpack (diag variant 3)
set -u
mkdir -p gpurun_out
C=${CASES:-mixed,sorted,uniform_768,uniform_769,mixed_x16}
timeout -k 10 200 python -u scripts/c3_probe.py $C > gpurun_out/c3.log 2>&1 && \
timeout -k 10 200 python -u scripts/c3_probe.py $C 3 >> gpurun_out/c3.log 2>&1
rc=$?
cat gpurun_out/c3.log | grep -v "amdgpu.ids"
exit $rc
