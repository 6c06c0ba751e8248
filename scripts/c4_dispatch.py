"""Per-dispatch durations of the analytics kernels in a rocprofv3 kernel trace (csv): the first
and the last full flow_reduce of c4_only.py (full config, then the rank-share runs)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
seq = []
for r in rows:
    k = r["Kernel_Name"]
    if "flow_" in k and "flowtab" not in k:
        seq.append((k.split("(")[0].replace("mgenx::", ""), int(r["Grid_Size_X"]),
                    (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
for x in seq[:12] + [("...", 0, 0.0)] + seq[-12:]:
    print(f"{x[0]:24s} {x[1]:9d} {x[2]:8.1f} us")
