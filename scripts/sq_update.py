"""SQ counters of the config-4 update kernel dispatches (rocprofv3 --pmc csv): per dispatch,
instructions per wave and the cycle split (SQ_*_CYCLES count quad-cycles on gfx950)."""
import csv
import glob
import sys
from collections import defaultdict

f = glob.glob(f"{sys.argv[1]}/**/*counter_collection.csv", recursive=True)
rows = list(csv.DictReader(open(f[0])))
by = defaultdict(dict)
for r in rows:
    if "flow_update_kernel" not in r["Kernel_Name"]:
        continue
    by[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
for d, c in list(by.items())[:3] + list(by.items())[-2:]:
    w = max(c.get("SQ_WAVES", 1), 1)
    print(d, {k: round(v / w, 1) if k != "SQ_WAVES" else v for k, v in sorted(c.items())})
