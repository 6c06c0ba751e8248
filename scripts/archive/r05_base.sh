#!/bin/bash
# Round 5 baseline on a fresh box: the whole -m gpu suite, the default bench line, a
# headline-only kernel trace (bench --no-extras), and the config-4 kernel trace (full + rank share).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  tail -${TAILN:-6} "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "STEP $name FAILED rc=$rc"; exit $rc; fi
}
step bar 60 ./scripts/diag/bar_probe 3000
step suite 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step bench 600 python -u bench.py
step headprof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/headprof -o head -- python3 -u bench.py --no-extras --no-cpu-baseline --steps 50 --warmup 10
step c4prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c4prof -o c4 -- python3 -u scripts/c4_only.py
python3 scripts/c4_dispatch.py gpurun_out/c4prof/c4_kernel_trace.csv
