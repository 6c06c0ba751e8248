#!/bin/bash
# general unpack kernel ablations (diag build): 3 = product general kernel unsorted,
# 1 = loads + XOR only, 2 = lookups on one L1-resident row
set -u
mkdir -p gpurun_out
C=${CASES:-uniform_768,mixed}
: > gpurun_out/c3abl.log
for v in 3 1 2; do
  timeout -k 10 200 python -u scripts/c3_probe.py $C $v >> gpurun_out/c3abl.log 2>&1 || exit $?
done
grep -v amdgpu.ids gpurun_out/c3abl.log
