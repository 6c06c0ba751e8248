#!/bin/bash
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
TESTS="tests/test_gpu_analytics.py tests/test_gpu_comm.py tests/test_compat_gpu.py" bash scripts/gpu_tests.sh || exit $?
timeout -k 10 300 python - <<'PY' > gpurun_out/c4.log 2>&1
import sys, json, torch
sys.path.insert(0, ".")
import bench
from mgen_amd import Engine
eng = Engine(0)
print(json.dumps(bench.extra_config4(torch, eng, torch.device("cuda:0"), 1, 0, None)))
PY
echo "c4 rc=$?"; tail -3 gpurun_out/c4.log
