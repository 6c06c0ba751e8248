"""Config-4 HBM traffic from rocprofv3 --pmc CSVs (scripts/pmc_c4.sh over traffic_c4.py).

FETCH_SIZE is calibrated PER ACCESS SHAPE: the probe reads 768 MiB coalesced at 4, 8, 16 and
24 bytes per lane; factor_w = bytes read / raw FETCH_SIZE bytes of that probe, and each kernel's
raw FETCH is scaled by the factor of its dominant access shape (listed per kernel).  WRITE_SIZE
is taken as exact (MI355X_MICROARCH.md: exact for 16-B-per-lane streaming stores; the config-4
kernels store 4-32 B per lane -- stated, not calibrated).  Durations: the median kernel-trace
time of the same launches in an unprofiled pass.  Writes profiles/r04/traffic_config4.json."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

out_dir = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
PROBE = 3 << 28  # bytes per calibration read


def load(counter):
    vals = defaultdict(list)
    for f in glob.glob(f"{out_dir}/pmc4_{counter}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if row.get("Counter_Name") == counter:
                vals[row["Kernel_Name"]].append(float(row["Counter_Value"]))
    return vals


def durations():
    vals = defaultdict(list)
    for f in glob.glob(f"{out_dir}/pmc4_time/**/*kernel_trace.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            vals[row["Kernel_Name"]].append(
                (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1000.0)
    return vals


def med(v):
    v = sorted(v)
    return v[len(v) // 2] if v else None


fetch, write, dur = load("FETCH_SIZE"), load("WRITE_SIZE"), durations()


def find(d, pat):
    ks = [k for k in d if pat in k]
    return ks


factors = {}
for w, pat in ((4, "stream_read_w_kernel<unsigned int>"), (8, "stream_read_w_kernel<HIP_vector_type"),
               (24, "stream_read_w_kernel<mgenx::SrW24>"), (16, "stream_read_kernel")):
    ks = find(fetch, pat)
    if ks:
        factors[w] = PROBE / (med(fetch[ks[0]]) * 1024)
n = int(open(os.path.join(out_dir, "traffic_c4_n.txt")).read())
F = 1024
T = (n + 4095) // 4096
H = (F + 1) * T * 4
# kernel -> (name pattern, access shape, algorithmic read bytes, algorithmic write bytes);
# launches in order of appearance: the column path first, then the rows pipeline
plan = [
    ("flow_hist_kernel", 4, n * 4, H),
    ("flow_colpart_kernel", 4, H, (F + 1) * 4 * ((T + 63) // 64)),
    ("flow_colbase_kernel", 4, 2 * (F + 1) * 4 * ((T + 63) // 64), (F + 1) * 4 * ((T + 63) // 64)),
    ("flow_colscan_kernel", 4, H + (F + 1) * 4 * ((T + 63) // 64), H),
    ("flow_order_kernel", 4, n * 26 + H, n * 24),
    ("flow_seg_kernel", 24, n * 24, n * 8),
    ("flow_update_kernel", 24, n * 24, n * 8),
    ("flow_chain_kernel", 8, n * 8, 0),
    ("unpack_fixed_kernel<4", 16, n * 64, n * 32),
    ("flowtab_insert_kernel", 16, n * (32 + 20), n * 4),
]
SMALL = ("flowtab_first", "flowtab_offsets", "flowtab_number", "flowtab_resolve",
         "flowtab_commit", "flow_init", "flow_long")
out = {"records": n, "flows": F, "fetch_factor_per_shape": {str(k): round(v, 4) for k, v in factors.items()},
       "note": __doc__.split("\n\n")[1].replace("\n", " "), "kernels": {}}
ROWS_ALGO = {"flow_order_kernel": (n * (32 + 8 + 4) + H, n * 24)}  # rows path: row + rx + index


def parts(k, vals):
    """(label, values): a kernel launched by both paths (6 launches) is split in dispatch order."""
    v = vals.get(k, [])
    if "flow_order_kernel<" in k:  # templated on the source: one name per path
        return [("rows" if "<true>" in k else "columns", v)]
    if len(v) >= 6 and k.startswith("mgenx::flow_"):
        h = len(v) // 2
        return [("columns", v[:h]), ("rows", v[h:])]
    return [("", v)]


for pat, w, ar0, aw0 in plan:
    for k in find(fetch, pat):
      for (lab, fv), (_, wv), (_, tv) in zip(parts(k, fetch), parts(k, write), parts(k, dur) if dur.get(k) else [("", [])] * 2):
        ar, aw = ar0, aw0
        name = k.split("(")[0]
        base = name.split("::")[-1].split("<")[0]
        if lab == "rows" and base in ROWS_ALGO:
            ar, aw = ROWS_ALGO[base]
        fr = med(fv)
        wr = med(wv) or 0.0
        t = med(tv)
        f = factors.get(w)
        rd = int(fr * 1024 * f) if f else None
        e = {"launches": len(fv), "shape_bytes_per_lane": w, "fetch_kb_raw": fr,
             "read_bytes": rd, "write_bytes": int(wr * 1024), "time_us": t}
        e["algorithmic_read"] = ar
        e["algorithmic_write"] = aw
        if rd is not None:
            e["read_ratio"] = round(rd / ar, 3) if ar else None
            e["write_ratio"] = round(int(wr * 1024) / aw, 3) if aw else None
        if t:
            e["algorithmic_TBps"] = round((ar + aw) / (t * 1e-6) / 1e12, 3)
        out["kernels"][name.replace("void ", "").split("<")[0] + (" [" + lab + "]" if lab else "")] = e
# the small steps (FindFlow numbering, flow init): raw counters and times only
for k in fetch:
    if any(x in k for x in SMALL):
        out["kernels"][k.split("(")[0]] = {"launches": len(fetch[k]), "fetch_kb_raw": med(fetch[k]),
                                           "write_kb": med(write.get(k, [0.0])),
                                           "time_us": med(dur.get(k, [])), "note": "small step"}
os.makedirs("profiles/r04", exist_ok=True)
json.dump(out, open("profiles/r04/traffic_config4.json", "w"), indent=1)
json.dump(out, open(f"{out_dir}/traffic_config4.json", "w"), indent=1)
print(json.dumps(out, indent=1)[:4000])
