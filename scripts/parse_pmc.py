"""Turn rocprofv3 --pmc CSVs into per-launch HBM bytes for the bench kernels.

gfx950 correction (MI355X_MICROARCH.md HBM section): FETCH_SIZE counts 64 B per
128-B request of a wide coalesced streaming read, i.e. reports 1/2 of the bytes; it is
doubled here.  WRITE_SIZE is exact for 16-B-per-lane streaming stores.  Units: KB.
Writes profiles/traffic_<ROUND>.json keyed by bench workload.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

out_dir = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
ROUND = os.environ.get("ROUND", "r02")


def load(counter):
    vals = defaultdict(list)
    for f in glob.glob(f"{out_dir}/pmc_{counter}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if row.get("Counter_Name") != counter:
                continue
            vals[row["Kernel_Name"]].append(float(row["Counter_Value"]))
    return vals


fetch, write = load("FETCH_SIZE"), load("WRITE_SIZE")
res = {}
for k in sorted(set(fetch) | set(write)):
    if "mgenx" not in k:
        continue
    f = sorted(fetch.get(k, [0.0]))
    w = sorted(write.get(k, [0.0]))
    fm, wm = f[len(f) // 2], w[len(w) // 2]
    res[k] = {"fetch_kb_raw": fm, "write_kb": wm, "launches": len(f),
              "hbm_bytes_per_launch": int(2 * fm * 1024 + wm * 1024)}
    print(k, res[k])
SLAB = 1073741824
algo = SLAB + 1048576 * 32


def find(pat):
    for k, v in res.items():
        if pat in k:
            return v
    return None


out = {"note": ("median over launches (each after a 512 MiB flush > Infinity Cache).  "
                "FETCH_SIZE is calibrated per access shape (MI355X_MICROARCH.md: only wide "
                "coalesced streaming reads are known to tally 1/2): the stream read shows "
                "the guide's factor, and mgenx_diag_group_rw mode 0, which reads exactly the "
                "1 GiB slab in the unpack's own access shape, calibrates that shape.  "
                "WRITE_SIZE is taken as exact."),
       "kernels": res}
sr = find("stream_read_kernel")
g0 = find("group_rw_kernel<0>")
rows = find("unpack_fixed_ring_kernel<16")
cols = find("unpack_fixed_kernel<16, 0, false, true>")
if sr:
    out["stream_read_fetch_factor"] = round(SLAB / (sr["fetch_kb_raw"] * 1024), 4)
if g0:
    factor = SLAB / (g0["fetch_kb_raw"] * 1024)
    out["unpack_shape_fetch_factor"] = round(factor, 4)
    for key, k in (("unpack_crc_1M_x_1024B", rows), ("unpack_crc_1M_x_1024B_columns", cols)):
        if k:
            hbm = int(k["fetch_kb_raw"] * 1024 * factor + k["write_kb"] * 1024)
            out[key] = {"hbm_bytes_per_launch": hbm, "algorithmic_bytes": algo,
                        "ratio": round(hbm / algo, 4),
                        "read_bytes": int(k["fetch_kb_raw"] * 1024 * factor),
                        "write_bytes": int(k["write_kb"] * 1024)}
# config 4: profiles/r04/traffic_config4.json (scripts/pmc_c4.sh: FETCH calibrated per access
# shape, per kernel algorithmic bytes)
out["config4"] = "profiles/r04/traffic_config4.json"
os.makedirs("profiles", exist_ok=True)
json.dump(out, open(f"profiles/traffic_{ROUND}.json", "w"), indent=1)
json.dump(out, open(f"{out_dir}/traffic_{ROUND}.json", "w"), indent=1)   # merged back by gpurun
print(json.dumps({k: v for k, v in out.items() if k != "kernels"}))
