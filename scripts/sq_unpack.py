"""SQ-counter probe (run under rocprofv3 --pmc ...): the config-3 unpack (unpack_var_kernel,
1M records U{64..1472} back to back -> 32-B rows) and the config-2 headline unpack
(unpack_fixed_ring_kernel, 1M x 1024 B -> rows), 3 launches each."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mgen_amd import PACK_CHECKSUM, Engine, to_device  # noqa: E402
from mgen_amd.workloads import udp_fixed, udp_mixed  # noqa: E402

N = 1 << 20
eng = Engine(0)
tmpl, pool, desc, offs, sizes = udp_mixed(N, 64, 1472, 64,
                                          payload_hex="00112233445566778899aabbccddeeff")
total = int(offs[-1] + sizes[-1])
d_tmpl, d_pool, d_desc = to_device(tmpl), to_device(pool), to_device(desc)
d_offs = to_device(offs).view(torch.int64)
d_len = to_device(sizes).view(torch.int32)
crc = torch.empty(len(tmpl), dtype=torch.int32, device="cuda")
eng.pack_prepare(d_tmpl, len(tmpl), d_pool, crc)
slab = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
eng.pack(d_tmpl, crc, d_desc, N, d_pool, slab, rec_off=d_offs, opts=PACK_CHECKSUM)
rows = {"rows": eng.alloc_rows(N)}
for _ in range(3):
    eng.unpack(slab, N, rec_off=d_offs, rec_len=d_len, cols=rows)
torch.cuda.synchronize()
del slab
t2, p2, de2 = udp_fixed(N, 1024)
dt, dp = to_device(t2), to_device(p2)
c2 = torch.empty(len(t2), dtype=torch.int32, device="cuda")
eng.pack_prepare(dt, len(t2), dp, c2)
slab2 = torch.empty(N * 1024, dtype=torch.uint8, device="cuda")
eng.pack(dt, c2, to_device(de2), N, dp, slab2, stride=1024, opts=PACK_CHECKSUM)
for _ in range(3):
    eng.unpack(slab2, N, stride=1024, fixed_len=1024, cols=rows)
torch.cuda.synchronize()
print("sq probe done")
