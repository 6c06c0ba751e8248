#!/bin/bash
# Round 4: the workgroup-per-flow analytics path -- parity tests, config-4 timing (product),
# the diagnostics build's seg off / on and order-phase timing, seg-kernel phase stamps.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  tail -${TAILN:-15} "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "STEP $name FAILED rc=$rc"; exit $rc; fi
}
step an_tests 600 python -u -m pytest tests/test_gpu_analytics.py -m gpu -x -q --timeout 120 --timeout-method thread
step c4 180 python -u scripts/c4_only.py
step ocut 600 python -u scripts/an_ocut.py
step segprof 300 python -u scripts/seg_prof.py
