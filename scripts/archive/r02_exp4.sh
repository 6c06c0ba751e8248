#!/bin/bash
set -u
mkdir -p gpurun_out
(rocm-smi --showserial --showuniqueid > gpurun_out/smi.log 2>&1 || true)
grep -i "serial\|unique" gpurun_out/smi.log | head -3
SWEEP_NAMES=${SWEEP_NAMES:-grw0,grw1,grw4096,grw4100,grw4112,grw4116,grw4101,grw4117,grw4132,r0,r1028,r1284} \
  timeout -k 10 300 python scripts/sweep_unpack.py > gpurun_out/sweep4.log 2>&1
rc=$?; echo "sweep rc=$rc"; tail -2 gpurun_out/sweep4.log; exit $rc
