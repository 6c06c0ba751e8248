#!/bin/bash
# Round 3: targeted GPU tests, the bench (no CPU leg), then kernel traces of config 4 and
# config 5 alone.  Any failure ends the script before the next GPU step.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  tail -${TAILN:-6} "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "STEP $name FAILED rc=$rc"; exit $rc; fi
  if grep -q -i "memory access fault\|core dumped\|illegal memory" "gpurun_out/$name.log"; then
    echo "FATAL: GPU error in $name"; exit 3; fi
}
if [ -n "${TESTS:-}" ]; then
  step tests 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 200 --timeout-method thread
fi
if [ "${BENCH:-1}" = "1" ]; then
  step bench 600 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline ${BENCH_ARGS:-}
fi
for c in ${TRACE:-}; do
  step trace_$c 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tr_$c -o tr \
      -- python3 -u scripts/${c}_only.py
  f=$(find gpurun_out/tr_$c -name "*kernel_stats.csv" | head -1)
  [ -n "$f" ] && cut -d, -f1-5 "$f" | head -14
done
