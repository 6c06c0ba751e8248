#!/bin/bash
# Order-kernel unit counters (config 4): TA / TCP / SQ, one rocprofv3 pass per group.
set -u
export TMPDIR=/tmp
OUT=gpurun_out
i=0
for grp in "TA_TA_BUSY_sum TA_FLAT_WRITE_WAVEFRONTS_sum GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD" \
           "TCP_TCC_WRITE_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum" \
           "TD_TD_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_INST_CYCLES_VMEM"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace --output-format csv \
      -d $OUT/pmco_$i -o p -- python3 scripts/c4_only.py > $OUT/pmco_$i.log 2>&1
  echo "pass $i rc=$?"
done
python3 - <<'PY'
import csv, glob, collections
for f in sorted(glob.glob("gpurun_out/pmco_*/**/*counter_collection.csv", recursive=True)):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "flow_order" in r.get("Kernel_Name", "") or "flow_update" in r.get("Kernel_Name", ""):
            k = ("order" if "flow_order" in r["Kernel_Name"] else "update", r["Counter_Name"])
            acc[k].append(float(r["Counter_Value"]))
    for k, v in sorted(acc.items()):
        print(f.split("/")[1], k, "n=%d" % len(v), "median=%.4g" % sorted(v)[len(v) // 2])
PY
