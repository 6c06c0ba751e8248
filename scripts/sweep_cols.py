"""Column placement vs the unpack kernel (config 2): the 14 core columns in separately
allocated torch buffers (as bench.py), in one buffer at 4 MiB-aligned offsets, and in one
buffer with column k skewed by k x (odd multiple of 128 B).  Interleaved rounds."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mgen_amd import COLS_CORE, PACK_CHECKSUM, Engine, to_device  # noqa: E402
from mgen_amd.workloads import udp_fixed  # noqa: E402

N, REC = 1 << 20, 1024
eng = Engine(0, diag=True)
tmpl, pool, desc = udp_fixed(N, REC)
d_tmpl, d_pool, d_desc = to_device(tmpl), to_device(pool), to_device(desc)
crc = torch.empty(len(tmpl), dtype=torch.int32, device="cuda")
eng.pack_prepare(d_tmpl, len(tmpl), d_pool, crc)
slab = torch.empty(N * REC, dtype=torch.uint8, device="cuda")
eng.pack(d_tmpl, crc, d_desc, N, d_pool, slab, stride=REC, opts=PACK_CHECKSUM)


def packed(skew):
    sizes = [np.dtype(dt).itemsize * w for _, dt, w in COLS_CORE]
    offs, o = [], 0
    for k, s in enumerate(sizes):
        offs.append(o)
        o += ((N * s + (4 << 20) - 1) // (4 << 20)) * (4 << 20) + k * skew
    buf = torch.empty(o + 4096, dtype=torch.uint8, device="cuda")
    cols = {}
    for (name, dt, w), off, s in zip(COLS_CORE, offs, sizes):
        cols[name] = buf[off:off + N * s].view(getattr(torch, dt))
    return cols, buf


layouts = {"torch": (eng.alloc_cols(N), None), "aligned4M": packed(0),
           "skew2176": packed(2176), "skew65664": packed(65536 + 128)}
res = {k: [] for k in layouts}
for rnd in range(5):
    for k, (cols, _) in layouts.items():
        eng.unpack(slab, N, stride=REC, fixed_len=REC, cols=cols)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(10):
            eng.unpack(slab, N, stride=REC, fixed_len=REC, cols=cols)
        b.record()
        torch.cuda.synchronize()
        res[k].append(a.elapsed_time(b) / 10)
for k, (cols, _) in layouts.items():
    assert int((cols["err"] != 0).sum()) == 0, k
print(json.dumps({k: round(float(np.median(v)), 4) for k, v in res.items()}))
print(json.dumps({k: [hex(t.data_ptr()) for t in v[0].values()][:4] for k, v in layouts.items()}))
