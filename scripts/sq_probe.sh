#!/bin/bash
# SQ counters (one rocprofv3 pass, kernel-trace only) over a probe script:
#   bash scripts/sq_probe.sh scripts/an_abl.py run   (PROBE args)
# prints the per-kernel medians of each counter.
set -u
export TMPDIR=/tmp
OUT=gpurun_out
CTRS=${CTRS:-"SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU"}
timeout -k 10 -s KILL 120 rocprofv3 --pmc $CTRS --kernel-trace --output-format csv \
    -d $OUT/sq_${TAG:-probe} -o sq -- python3 "$@" > $OUT/sq_${TAG:-probe}.log 2>&1
rc=$?; echo "rc=$rc"; tail -2 $OUT/sq_${TAG:-probe}.log
[ $rc -ne 0 ] && exit $rc
python3 - "$OUT/sq_${TAG:-probe}" <<'PY'
import csv, glob, collections, sys
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"][:50]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k, {c: round(sorted(v)[len(v) // 2]) for c, v in sorted(d.items())})
PY
