"""Pack timing on the config-2 batch (1M x 1024 B): checksum on/off, plus a plain 1 GiB fill
(the write roofline reference), interleaved rounds in one process."""
import json
import os
import sys

import numpy as np
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
out_len = torch.empty(N, dtype=torch.int32, device="cuda")


def run(name):
    eng.set_pack_variant(int(name[-1]) if name[-1].isdigit() else 0)
    name = name.rstrip("0123456789")
    if name == "pack_ck":
        eng.pack(d_tmpl, crc, d_desc, N, d_pool, slab, stride=REC, opts=PACK_CHECKSUM, out_len=out_len)
    elif name == "pack_nock":
        eng.pack(d_tmpl, crc, d_desc, N, d_pool, slab, stride=REC, opts=0, out_len=out_len)
    elif name == "fill":
        slab.fill_(7)


names = os.environ.get("SWEEP_NAMES", "pack_ck,pack_nock,fill").split(",")
res = {k: [] for k in names}
for rnd in range(5):
    for k in names:
        run(k)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(10):
            run(k)
        b.record()
        torch.cuda.synchronize()
        res[k].append(a.elapsed_time(b) / 10)
out = {k: {"ms": round(float(np.median(t)), 4),
           "GBps": round(N * REC / float(np.median(t)) / 1e6, 1)} for k, t in res.items()}
print(json.dumps(out))
