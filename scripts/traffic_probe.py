"""Kernels for the HBM-traffic counter passes (run under rocprofv3 --pmc ...), config 2 data,
3 launches each after a 512 MiB flush (> Infinity Cache): the plain stream read of the 1 GiB
slab, the unpack's read pattern alone (mgenx_diag_group_rw mode 0: exactly the slab bytes in
the unpack's own access shape -> FETCH_SIZE calibration for that shape), the product unpack
with 32-B row output (the bench headline), and the same with the SoA columns.  Then config 4's
receive pipeline on rows (8.4M 256-B datagrams: unpack -> FindFlow from the rows ->
mgenx_flow_reduce_rows), one flush before each pipeline run."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mgen_amd import PACK_CHECKSUM, Engine, to_device  # noqa: E402
from mgen_amd.workloads import udp_fixed  # noqa: E402

N, REC = 1 << 20, 1024
eng = Engine(0, diag=True)
tmpl, pool, desc = udp_fixed(N, REC)
d_tmpl, d_pool, d_desc = to_device(tmpl), to_device(pool), to_device(desc)
crc = torch.empty(len(tmpl), dtype=torch.int32, device="cuda")
eng.pack_prepare(d_tmpl, len(tmpl), d_pool, crc)
slab = torch.empty(N * REC, dtype=torch.uint8, device="cuda")
eng.pack(d_tmpl, crc, d_desc, N, d_pool, slab, stride=REC, opts=PACK_CHECKSUM)
cols = eng.alloc_cols(N)
rows = eng.alloc_rows(N)
probe = torch.empty(N * 32, dtype=torch.uint8, device="cuda")
flush = torch.empty(512 << 20, dtype=torch.uint8, device="cuda")
for _ in range(3):
    flush.fill_(1)
    eng.stream_read(slab, grid=2048)
    flush.fill_(1)
    eng.group_rw(slab, probe, 0)
    flush.fill_(1)
    eng.unpack(slab, N, stride=REC, fixed_len=REC, cols={"rows": rows})
    flush.fill_(1)
    eng.unpack(slab, N, stride=REC, fixed_len=REC, cols=cols)
torch.cuda.synchronize()
assert int((cols["err"] != 0).sum()) == 0
del cols, rows, probe, slab

# config 4 on rows
import numpy as np  # noqa: E402
from mgen_amd import DESC_DTYPE  # noqa: E402
from mgen_amd.workloads import make_templates, poisson_flows  # noqa: E402
NF, MSG = 1024, 256
d = poisson_flows(8 * N, NF, mean_gap_us=1000)
n = len(d["seq"])
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
rx_s = torch.from_numpy(d["rx_sec"]).cuda()
rx_u = torch.from_numpy(d["rx_usec"]).cuda()
fidx = torch.empty(n, dtype=torch.int32, device="cuda")
nf = torch.zeros(1, dtype=torch.int32, device="cuda")
table = eng.flow_table(2 * NF)
for _ in range(3):
    flush.fill_(1)
    eng.unpack(slab, n, stride=MSG, fixed_len=MSG, cols=rows)
    eng.flow_lookup(table, rows, src.reshape(-1), n, flow_idx=fidx, n_flows=nf)
    flows = eng.flow_init(NF, 1.0)
    eng.flow_reduce_rows(flows, NF, fidx, rows["rows"], rx_s, rx_u, n=n)
torch.cuda.synchronize()
assert int(nf.cpu()[0]) == NF
eng.flow_table_destroy(table)
os.makedirs("gpurun_out", exist_ok=True)
open("gpurun_out/traffic_probe_n4.txt", "w").write(str(n))
print("traffic probe done", n)
