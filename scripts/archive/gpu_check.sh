#!/bin/bash
# One gpurun call: GPU tests, smoke, bench, rocprof kernel trace.  Each GPU step has its
# own time limit; a fault / abort / timeout (exit >= 124 or signal) ends the script there.
# Ordinary test failures (exit 1) do not stop the later measurement steps.
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # step <name> <timeout-seconds> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 30 $OUT/$name.log
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
    echo "FATAL: $name rc=$rc -- stopping"; exit $rc
  fi
  return 0
}
python -c "import __graft_entry__ as g; g.build()" > $OUT/build.log 2>&1 || { cat $OUT/build.log; exit 1; }
step pytest_gpu 600 python -m pytest tests -m gpu -x -q ${PYTEST_ARGS:-}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py --steps ${STEPS:-50} --warmup ${WARMUP:-10}
if [ "${PROFILE:-1}" = "1" ]; then
  step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline
  find $OUT/prof -name "*stats*" | head
fi
