"""Kernels for config 4's HBM-traffic counter passes (run under rocprofv3 --pmc ...), each
after a 512 MiB flush (> Infinity Cache): the FETCH_SIZE calibration reads -- 1 GiB read
coalesced at 4, 8, 16 and 24 bytes per lane (the access shapes of the config-4 kernels) --
then mgenx_flow_reduce over config 4's columns (8.4M records, 1024 flows), and the rows
pipeline (header-only unpack of 256-B datagrams -> FindFlow -> flow_reduce_rows)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mgen_amd import DESC_DTYPE, Engine, to_device  # noqa: E402
from mgen_amd.workloads import make_templates, poisson_flows  # noqa: E402

eng = Engine(0, diag=True)
flush = torch.empty(512 << 20, dtype=torch.uint8, device="cuda")
buf = torch.ones(3 << 28, dtype=torch.uint8, device="cuda")  # 768 MiB: a multiple of 4, 8, 16, 24
for _ in range(3):
    for w in (4, 8, 24):
        flush.fill_(1)
        eng.stream_read_w(buf, w)
    flush.fill_(1)
    eng.stream_read(buf)
torch.cuda.synchronize()
del buf

NF = 1024
d = poisson_flows(8388608, NF, mean_gap_us=1000)
n = len(d["seq"])
t = {k: torch.from_numpy(v).cuda() for k, v in d.items()}
idx = torch.from_numpy((d["flow_id"] - 1).astype(np.uint32)).cuda()
for _ in range(3):
    flush.fill_(1)
    flows = eng.flow_init(NF, 1.0)
    eng.flow_reduce(flows, NF, idx, t["seq"], t["tx_sec"], t["tx_usec"], t["msg_len"],
                    t["rx_sec"], t["rx_usec"], n=n)
torch.cuda.synchronize()

MSG = 256
tmpl, pool = make_templates(NF)
desc = np.zeros(n, DESC_DTYPE)
desc["tmpl"], desc["seq_num"] = d["flow_id"] - 1, d["seq"]
desc["tx_sec"], desc["tx_usec"], desc["msg_len"] = d["tx_sec"], d["tx_usec"], MSG
dt, dp = to_device(tmpl), to_device(pool)
crc = torch.empty(NF, dtype=torch.int32, device="cuda")
eng.pack_prepare(dt, NF, dp, crc)
slab = torch.empty(n * MSG, dtype=torch.uint8, device="cuda")
eng.pack(dt, crc, to_device(desc), n, dp, slab, stride=MSG)
rows = {"rows": eng.alloc_rows(n)}
fid = torch.from_numpy(d["flow_id"].astype(np.int64)).cuda()
src = torch.zeros(n, 20, dtype=torch.uint8, device="cuda")
src[:, 0], src[:, 1], src[:, 2], src[:, 3], src[:, 4] = 1, 4, 0x89, 0x13, 10
src[:, 6], src[:, 7] = ((fid >> 8) & 255).to(torch.uint8), (fid & 255).to(torch.uint8)
fidx = torch.empty(n, dtype=torch.int32, device="cuda")
nf = torch.zeros(1, dtype=torch.int32, device="cuda")
table = eng.flow_table(2 * NF)
for _ in range(3):
    flush.fill_(1)
    eng.unpack(slab, n, stride=MSG, fixed_len=MSG, cols=rows)
    eng.flow_lookup(table, rows, src.reshape(-1), n, flow_idx=fidx, n_flows=nf)
    flows = eng.flow_init(NF, 1.0)
    eng.flow_reduce_rows(flows, NF, fidx, rows["rows"], t["rx_sec"], t["rx_usec"], n=n)
torch.cuda.synchronize()
assert int(nf.cpu()[0]) == NF
eng.flow_table_destroy(table)
os.makedirs("gpurun_out", exist_ok=True)
open("gpurun_out/traffic_c4_n.txt", "w").write(str(n))
print("traffic c4 probe done", n)
