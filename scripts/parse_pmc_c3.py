"""Config-3 counter passes -> profiles/<ROUND>/traffic_config3.json (per-launch HBM bytes of
the pack and the variable-length unpack against their algorithmic bytes).  FETCH_SIZE is
scaled by the factor the plain stream read of the same slab shows (MI355X_MICROARCH.md:
wide coalesced reads tally 1/2); WRITE_SIZE is taken as exact."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

import numpy as np

out_dir = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
ROUND = os.environ.get("ROUND", "r02")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mgen_amd.workloads import udp_mixed  # noqa: E402

N = 1 << 20
_, _, _, offs, sizes = udp_mixed(N, 64, 1472, 64, payload_hex="00112233445566778899aabbccddeeff")
SLAB = int(offs[-1] + sizes[-1])
SLAB_ALLOC = (SLAB + 4095) // 4096 * 4096


def load(counter):
    vals = defaultdict(list)
    for f in glob.glob(f"{out_dir}/pmc_{counter}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if row.get("Counter_Name") == counter:
                vals[row["Kernel_Name"]].append(float(row["Counter_Value"]))
    return vals


fetch, write = load("FETCH_SIZE"), load("WRITE_SIZE")
med = {}
for k in set(fetch) | set(write):
    if "mgenx" in k:
        f, w = sorted(fetch.get(k, [0.0])), sorted(write.get(k, [0.0]))
        med[k] = (f[len(f) // 2] * 1024, w[len(w) // 2] * 1024, len(f))


def find(pat):
    return next((v for k, v in med.items() if pat in k), None)


sr, pk, up = find("stream_read_kernel"), find("pack_kernel"), find("unpack_var_kernel")
factor = SLAB_ALLOC / sr[0] if sr else 2.0
out = {"note": __doc__.strip(), "records": N, "slab_bytes": SLAB,
       "stream_read_fetch_factor": round(factor, 4), "kernels": {}}
algo = {"pack_kernel": (N * 20 + N * 16, SLAB), "unpack_var_kernel": (SLAB + N * 12, N * 32)}
for name, v in (("pack_kernel", pk), ("unpack_var_kernel", up)):
    if v is None:
        continue
    rd, wr = int(v[0] * factor), int(v[1])
    ar, aw = algo[name]
    out["kernels"][name] = {"read_bytes": rd, "write_bytes": wr, "hbm_bytes": rd + wr,
                            "fetch_raw_bytes": int(v[0]), "launches": v[2],
                            "algorithmic_read": ar, "algorithmic_write": aw,
                            "ratio": round((rd + wr) / (ar + aw), 4)}
os.makedirs(f"profiles/{ROUND}", exist_ok=True)
json.dump(out, open(f"profiles/{ROUND}/traffic_config3.json", "w"), indent=1)
json.dump(out, open(f"{out_dir}/traffic_config3.json", "w"), indent=1)  # merged back by gpurun
print(json.dumps(out, indent=1))
