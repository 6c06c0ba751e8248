"""Per-call timeline of the whole-stream scans in a rocprofv3 kernel trace (each call starts
at a detect launch): kernel, start and end in us from the call's first launch."""
import csv
import glob
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/scanprof"
path = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "scan_detect" in r["Kernel_Name"]]
spans = []
for n, j in enumerate(idx):
    t0 = int(rows[j]["Start_Timestamp"])
    k, last = j, t0
    stop = idx[n + 1] if n + 1 < len(idx) else len(rows)
    lines = []
    while k < stop:
        r = rows[k]
        s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
        lines.append(f"  {r['Kernel_Name'][:60]:60s} {s / 1e3:8.1f} {e / 1e3:8.1f} {(e - s) / 1e3:6.1f}")
        last = max(last, int(r["End_Timestamp"]))
        k += 1
    spans.append((last - t0) / 1e3)
    if n >= len(idx) - 2:
        print("\n".join(lines))
        print()
spans.sort()
print("calls", len(spans), "GPU span per call: median %.1f us, min %.1f" % (spans[len(spans) // 2], spans[0]))
