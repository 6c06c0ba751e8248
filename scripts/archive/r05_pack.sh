#!/bin/bash
# Round 5: pack store phase -- pack parity tests, then the bench line (pack_ms, config-3 pack,
# tcp_tx) without the CPU leg.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  tail -${TAILN:-3} "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "STEP $name FAILED rc=$rc"; exit $rc; fi
}
step pack_tests 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pack_layout.py tests/test_gpu_pack_msgs.py tests/test_gpu_tcp_tx.py -m gpu -x -q --timeout 120 --timeout-method thread
step bench_nocpu 300 python -u bench.py --no-cpu-baseline
python3 - <<'PY'
import json
l=[x for x in open("gpurun_out/bench_nocpu.log") if x.startswith("{")][-1]
d=json.loads(l); e=d["extra"]
print(json.dumps({"value": d["value"], "pack_ms": e["pack_ms"], "c3": e["config3_mixed_pack_unpack"], "tcp_tx_ms": e["config5_tcp_scan_unpack"]["tcp_tx_ms"], "scan_ms": e["config5_tcp_scan_unpack"]["scan_ms"], "c4": e["config4_flow_reduce"]["reduce_ms"], "share8": e["config4_flow_reduce"]["rank_share_at_8"]["reduce_ms"]}))
PY
