#!/bin/bash
# Unit counters of a plain 1 GiB fill (compare scripts/pmc_pack.sh).
set -u
export TMPDIR=/tmp
OUT=gpurun_out
i=0
for grp in "TA_TA_BUSY_sum TA_FLAT_WRITE_WAVEFRONTS_sum GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VMEM_WR" \
           "TCP_TCC_WRITE_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace --output-format csv \
      -d $OUT/pmcf_$i -o p -- python3 scripts/fill_probe.py > $OUT/pmcf_$i.log 2>&1
  echo "pass $i rc=$?"
done
timeout -k 10 60 python3 scripts/fill_probe.py
python3 - <<'PY'
import csv, glob, collections
for f in sorted(glob.glob("gpurun_out/pmcf_*/**/*counter_collection.csv", recursive=True)):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "Fill" in r.get("Kernel_Name", "") or "fill" in r.get("Kernel_Name", ""):
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in sorted(acc.items()):
        print(f.split("/")[1], k, "n=%d" % len(v), "median=%.4g" % sorted(v)[len(v) // 2])
PY
