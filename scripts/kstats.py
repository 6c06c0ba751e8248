"""Per-kernel summary of rocprofv3 --stats CSVs: python scripts/kstats.py <dir> [n]."""
import csv
import glob
import sys

for f in sorted(glob.glob(f"{sys.argv[1]}/**/*kernel_stats.csv", recursive=True)):
    print("==", f)
    for r in list(csv.DictReader(open(f)))[:int(sys.argv[2]) if len(sys.argv) > 2 else 16]:
        print(f'{r["Name"][:72]:72s} {r["Calls"]:>5s} {float(r["AverageNs"]) / 1e3:9.1f} us')
