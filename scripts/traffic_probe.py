"""Kernels for the HBM-traffic counter passes (run under rocprofv3 --pmc ...), config 2 data,
3 launches each after a 512 MiB flush (> Infinity Cache): the plain stream read of the 1 GiB
slab, the unpack's read pattern alone (mgenx_diag_group_rw mode 0: exactly the slab bytes in
the unpack's own access shape -> FETCH_SIZE calibration for that shape), the product unpack
with 32-B row output (the bench headline), and the same with the SoA columns.  (Config 4: scripts/traffic_c4.py.)"""
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

print("traffic probe done")
