"""Config 2 pack under diagnostics variants (argv: variants; default 0 10), interleaved twice:
0 = product, 10 = the meta waves never help the joint store."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mgen_amd import PACK_CHECKSUM, Engine, to_device  # noqa: E402
from mgen_amd.workloads import udp_fixed  # noqa: E402

n = 1 << 20
d = Engine(0, diag=True)
tmpl, pool, desc = udp_fixed(n, 1024)
dt, dp, dd = to_device(tmpl), to_device(pool), to_device(desc)
crc = torch.empty(len(tmpl), dtype=torch.int32, device="cuda")
d.pack_prepare(dt, len(tmpl), dp, crc)
slab = torch.empty(n * 1024, dtype=torch.uint8, device="cuda")
ol = torch.empty(n, dtype=torch.int32, device="cuda")
ref = None
for rnd in range(2):
    for v in [int(a) for a in sys.argv[1:]] or [0, 10]:
        d.set_pack_variant(v)
        f = lambda: d.pack(dt, crc, dd, n, dp, slab, stride=1024, opts=PACK_CHECKSUM, out_len=ol)  # noqa
        f()
        torch.cuda.synchronize()
        h = int(torch.sum(slab.view(torch.int64)[::4097]).item())
        ref = h if ref is None else ref
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(20):
            f()
        b.record()
        torch.cuda.synchronize()
        print(f"variant {v} config2 pack_ms {a.elapsed_time(b) / 20:.4f} same={h == ref}", flush=True)
