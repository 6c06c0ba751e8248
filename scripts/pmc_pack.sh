#!/bin/bash
# Config-2 pack unit counters (SQ / TA / TCP), one rocprofv3 pass per group, pack_meta_probe.py.
set -u
export TMPDIR=/tmp
OUT=gpurun_out
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" \
           "TA_TA_BUSY_sum TA_FLAT_WRITE_WAVEFRONTS_sum GRBM_GUI_ACTIVE" \
           "TCP_TCC_WRITE_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv \
      -d $OUT/pmcp_$i -o p -- python3 scripts/pack_meta_probe.py > $OUT/pmcp_$i.log 2>&1
  echo "pass $i rc=$?"
done
python3 - <<'PY'
import csv, glob, collections
for f in sorted(glob.glob("gpurun_out/pmcp_*/**/*counter_collection.csv", recursive=True)):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "pack_kernel<false>" in r.get("Kernel_Name", ""):
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in sorted(acc.items()):
        print(f.split("/")[1], k, "n=%d" % len(v), "median=%.4g" % sorted(v)[len(v) // 2])
PY
