#!/bin/bash
# round 6: config-3 var kernel with 64-B-aligned row loads (ablation, timing only)
set -u
export TMPDIR=/tmp
VARIANTS=0,33,20 FIXED=0 ROUNDS=5 timeout -k 10 600 python3 -u scripts/var_shapes.py || exit 1
