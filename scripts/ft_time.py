"""FindFlow (mgenx_flow_lookup) alone on config 4's records, columns and rows, as bench.py's
extra_config4 / pipeline_config4 key them; prints one JSON line.  With the diagnostics
library (MGENX_LIB_OVERRIDE=mgen_amd/libmgenx_diag.so) MGENX_FT_MODE picks an ablation of
the insert kernel (1: key loads + hash, 2: key loads only)."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from mgen_amd import DESC_DTYPE, Engine, to_device  # noqa: E402
from mgen_amd.workloads import make_templates, poisson_flows  # noqa: E402

eng = Engine(0)
dev = torch.device("cuda:0")
n_flows = 1024
d = poisson_flows(bench.N4_TOTAL, n_flows, mean_gap_us=1000)
n = len(d["flow_id"])
t = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in d.items()}
src = torch.zeros(n, 20, dtype=torch.uint8, device=dev)
fid = t["flow_id"]
f64 = fid.to(torch.int64)
src[:, 0], src[:, 1], src[:, 2], src[:, 3] = 1, 4, 0x89, 0x13
src[:, 4], src[:, 6], src[:, 7] = 10, ((f64 >> 8) & 255).to(torch.uint8), (f64 & 255).to(torch.uint8)
dst_addr = torch.zeros(n, 16, dtype=torch.uint8, device=dev)
dst_addr[:, 0], dst_addr[:, 3] = 127, 1
cols = {"dst_addr": dst_addr.reshape(-1), "flow_id": fid.view(torch.int32),
        "dst_len": torch.full((n,), 4, dtype=torch.uint8, device=dev),
        "dst_port": torch.full((n,), 5000, dtype=torch.int16, device=dev)}
out = {"records": n}
warm = eng.flow_table(2 * n_flows)   # (first launches, allocations)
eng.flow_lookup(warm, cols, src.reshape(-1), n)
torch.cuda.synchronize()
eng.flow_table_destroy(warm)
table = eng.flow_table(2 * n_flows)
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
fidx, nf = eng.flow_lookup(table, cols, src.reshape(-1), n)   # every key new in this call
b.record()
torch.cuda.synchronize()
out["cols_first_call_ms"] = round(a.elapsed_time(b), 4)
ok = int(nf.cpu()[0]) == len(np.unique(d["flow_id"]))
want = fidx.clone()
out["cols_ms"] = round(bench.timed(torch, lambda: eng.flow_lookup(table, cols, src.reshape(-1), n,
                                                                 flow_idx=fidx, n_flows=nf), 20), 4)
torch.cuda.synchronize()
out["cols_same"] = bool(ok and torch.equal(fidx, want))
eng.flow_table_destroy(table)
# rows: GPU-packed 256-B datagrams unpacked to 32-B rows
idx = (d["flow_id"] - 1).astype(np.uint32)
msg = 256
tmpl, pool = make_templates(n_flows)
desc = np.zeros(n, DESC_DTYPE)
desc["tmpl"], desc["seq_num"] = idx, d["seq"]
desc["tx_sec"], desc["tx_usec"], desc["msg_len"] = d["tx_sec"], d["tx_usec"], msg
dt, dp = to_device(tmpl, eng.device), to_device(pool, eng.device)
crc = torch.empty(n_flows, dtype=torch.int32, device=dev)
eng.pack_prepare(dt, n_flows, dp, crc)
slab = torch.empty(n * msg, dtype=torch.uint8, device=dev)
eng.pack(dt, crc, to_device(desc, eng.device), n, dp, slab, stride=msg)
rows = {"rows": eng.alloc_rows(n)}
eng.unpack(slab, n, stride=msg, fixed_len=msg, cols=rows)
table = eng.flow_table(2 * n_flows)
f2 = torch.empty(n, dtype=torch.int32, device=dev)
n2 = torch.zeros(1, dtype=torch.int32, device=dev)
eng.flow_lookup(table, rows, src.reshape(-1), n, flow_idx=f2, n_flows=n2)
torch.cuda.synchronize()
w2 = f2.clone()
out["rows_ms"] = round(bench.timed(torch, lambda: eng.flow_lookup(table, rows, src.reshape(-1), n,
                                                                 flow_idx=f2, n_flows=n2), 20), 4)
torch.cuda.synchronize()
out["rows_same"] = bool(torch.equal(f2, w2) and int(n2.cpu()[0]) == int(nf.cpu()[0]))
eng.flow_table_destroy(table)
out["mode"] = os.environ.get("MGENX_FT_MODE", "0")
out["gmul"] = os.environ.get("MGENX_FT_GMUL", "-")
out["kcap"] = os.environ.get("MGENX_FT_KCAP", "-")
out["lib"] = os.path.basename(os.environ.get("MGENX_LIB_OVERRIDE", "libmgenx.so"))
print(json.dumps(out))
