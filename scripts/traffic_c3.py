"""Kernels for the config-3 HBM-traffic counter passes (run under rocprofv3 --pmc ...):
1M records of U{64..1472} bytes packed back to back (bench.py extra_config3), 3 launches
each after a 512 MiB flush (> Infinity Cache): the plain stream read of the slab (FETCH_SIZE
calibration for wide coalesced reads), the product pack (checksum on) and the product
unpack (variable-length kernel, 32-B rows: the product layout)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mgen_amd import PACK_CHECKSUM, Engine, to_device  # noqa: E402
from mgen_amd.workloads import udp_mixed  # noqa: E402

N = 1 << 20
eng = Engine(0, diag=True)
tmpl, pool, desc, offs, sizes = udp_mixed(N, 64, 1472, 64,
                                          payload_hex="00112233445566778899aabbccddeeff")
total = int(offs[-1] + sizes[-1])
d_tmpl, d_pool, d_desc = to_device(tmpl), to_device(pool), to_device(desc)
d_offs = to_device(offs).view(torch.int64)
d_len = to_device(sizes).view(torch.int32)
crc = torch.empty(len(tmpl), dtype=torch.int32, device="cuda")
eng.pack_prepare(d_tmpl, len(tmpl), d_pool, crc)
slab = torch.empty((total + 4095) // 4096 * 4096, dtype=torch.uint8, device="cuda")
out_len = torch.empty(N, dtype=torch.int32, device="cuda")
cols = {"rows": eng.alloc_rows(N)}
flush = torch.empty(512 << 20, dtype=torch.uint8, device="cuda")
for _ in range(3):
    flush.fill_(1)
    eng.pack(d_tmpl, crc, d_desc, N, d_pool, slab, rec_off=d_offs, opts=PACK_CHECKSUM,
             out_len=out_len)
    flush.fill_(1)
    eng.stream_read(slab, grid=2048)
    flush.fill_(1)
    eng.unpack(slab, N, rec_off=d_offs, rec_len=d_len, cols=cols)
torch.cuda.synchronize()
assert int(((cols["rows"].view(torch.int32).view(N, 8)[:, 6] >> 24) & 0xFF).sum()) == 0
print(f"traffic probe config 3 done: {total} slab bytes")
