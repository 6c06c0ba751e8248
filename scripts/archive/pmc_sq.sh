#!/bin/bash
# SQ counters for the unpack ablation modes (one counter pass, kernel-trace only).
set -u
export TMPDIR=/tmp
OUT=gpurun_out
CTRS=${CTRS:-"SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU"}
timeout -k 10 300 rocprofv3 --pmc $CTRS --kernel-trace --output-format csv \
    -d $OUT/pmc_sq -o sq -- python scripts/sweep_unpack.py > $OUT/pmc_sq.log 2>&1
rc=$?; echo "rc=$rc"; tail -3 $OUT/pmc_sq.log
python - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/pmc_sq/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k, {c: round(sorted(v)[len(v)//2]) for c, v in d.items()})
PY
