#!/bin/bash
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
(rocm-smi --showuniqueid > gpurun_out/smi.log 2>&1 || true); grep -i "unique id" gpurun_out/smi.log | tail -1
bash scripts/gpu_tests.sh || exit $?
SWEEP_NAMES=${SWEEP_NAMES:-grw0,grw1,r0,r13,r1028,r1284} \
  timeout -k 10 300 python scripts/sweep_unpack.py > gpurun_out/sweep8.log 2>&1 || { echo "sweep failed"; tail -5 gpurun_out/sweep8.log; exit 4; }
tail -1 gpurun_out/sweep8.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench8.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/bench8.log; exit 5; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/bench8.log").read().strip().splitlines()[-1])
print("value", d["value"], "roofline", d["roofline"])
e = d["extra"]
print({k: e[k] for k in e if not isinstance(e[k], dict)})
print("config4", e.get("config4_flow_reduce"))
PY
