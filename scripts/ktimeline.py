"""Print one rocprofv3 kernel_stats.csv (name, calls, average us) and, with a trace csv, the
last N kernels' timeline.  Usage: python scripts/ktimeline.py stats.csv [trace.csv [N]]"""
import csv
import sys

for r in csv.DictReader(open(sys.argv[1])):
    print(f"{r['Name'][:64]:64s} {r['Calls']:>6s} {float(r['AverageNs']) / 1e3:9.1f} us")
if len(sys.argv) > 2:
    tr = sorted(csv.DictReader(open(sys.argv[2])), key=lambda r: int(r['Start_Timestamp']))
    k = int(sys.argv[3]) if len(sys.argv) > 3 else 12
    t0 = int(tr[-k]['Start_Timestamp'])
    for r in tr[-k:]:
        s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
        print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  {r['Kernel_Name'][:56]}")
