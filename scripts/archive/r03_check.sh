#!/bin/bash
# Round 3 GPU check: the named test files first (verbose), then the whole -m gpu suite, then
# a short bench.  Any fault / abort / timeout ends the script before the next GPU step.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  tail -25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "STEP $name FAILED rc=$rc"; exit $rc; fi
  if grep -q -i "memory access fault\|core dumped\|illegal memory" "gpurun_out/$name.log"; then
    echo "FATAL: GPU error in $name"; exit 3; fi
}
if [ -n "${FIRST:-}" ]; then
  step first 600 python -u -m pytest $FIRST -m gpu -x -v --timeout 300 --timeout-method thread
fi
if [ "${SUITE:-1}" = "1" ]; then
  step suite 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
fi
if [ "${BENCH:-1}" = "1" ]; then
  step bench 600 python -u bench.py --steps ${STEPS:-20} --warmup 5 ${BENCH_ARGS:-}
fi
