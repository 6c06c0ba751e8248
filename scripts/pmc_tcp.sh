# HBM traffic of config 5's TCP transmit: FETCH_SIZE and WRITE_SIZE in passes of their own
# (kernel-trace only), over scripts/tcp_time.py; per-launch averages per kernel
set -u
export TMPDIR=/tmp
OUT=gpurun_out
for c in FETCH_SIZE WRITE_SIZE; do
  rm -rf $OUT/pmctcp_$c
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv \
      -d $OUT/pmctcp_$c -o pmc -- python3 scripts/tcp_time.py > $OUT/pmctcp_$c.log 2>&1
  rc=$?
  echo "pmc $c rc=$rc"; tail -n 1 $OUT/pmctcp_$c.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
python3 - <<'PY'
import csv, glob, collections
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    f = glob.glob(f"gpurun_out/pmctcp_{c}/**/*counter_collection.csv", recursive=True)
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f[0])):
        acc[r["Kernel_Name"][:48]].append(float(r["Counter_Value"]))
    for k, v in acc.items():
        if "tcp_plan0" in k or "pack_kernel" in k:
            print(c, k, "launches", len(v), "avg KB", round(sum(v) / len(v), 1))
PY
