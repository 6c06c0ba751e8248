#!/bin/bash
# Store-placement probes: group_rw with row stores buffered K groups (K = 1..16) under three
# store policies, and end-of-wave burst ablations of the headline kernel.
set -u
mkdir -p gpurun_out
SWEEP_NAMES=${SWEEP_NAMES:-grw0,grw1,grw16,grw32,grw48,grw64,grw80,grw304,grw336,grw560,grw592,r0,r1028,r1284,r1300,r1348,r1812,fill_rows} \
  timeout -k 10 300 python scripts/sweep_unpack.py > gpurun_out/sweep2.log 2>&1
rc=$?; echo "sweep rc=$rc"; tail -3 gpurun_out/sweep2.log; exit $rc
