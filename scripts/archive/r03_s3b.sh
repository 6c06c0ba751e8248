#!/bin/bash
# scan tests (pruning), config-5 scan timing, var-kernel A/B (interleaved)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  tail -${TAILN:-15} "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "STEP $name FAILED rc=$rc"; exit $rc; fi
}
step scan_tests 400 python -u -m pytest tests/test_gpu_scan.py -m gpu -x -q --timeout 200 --timeout-method thread
step c5 120 python -u scripts/c5_only.py
TAILN=12 step var 300 env VARIANTS=0,21,20 ROUNDS=7 FIXED=0 python -u scripts/var_shapes.py
