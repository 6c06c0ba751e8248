"""Kernels for the HBM-traffic counter passes (run under rocprofv3 --pmc ...): the plain
16-B/lane stream read of the 1 GiB slab (the guide's calibrated shape), the fixed-length
unpack (product), its loads-only ablation (mode 5: exactly the slab bytes in the unpack's
own access shape -> calibration of FETCH_SIZE for that shape), the general kernel and the
header-only decode, 3 launches each, config 2 data."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mgen_amd import OPT_SKIP_CRC, PACK_CHECKSUM, Engine, to_device  # noqa: E402
from mgen_amd.workloads import udp_fixed  # noqa: E402

N, REC = 1 << 20, 1024
eng = Engine(0)
tmpl, pool, desc = udp_fixed(N, REC)
d_tmpl, d_pool, d_desc = to_device(tmpl), to_device(pool), to_device(desc)
crc = torch.empty(len(tmpl), dtype=torch.int32, device="cuda")
eng.pack_prepare(d_tmpl, len(tmpl), d_pool, crc)
slab = torch.empty(N * REC, dtype=torch.uint8, device="cuda")
eng.pack(d_tmpl, crc, d_desc, N, d_pool, slab, stride=REC, opts=PACK_CHECKSUM)
cols = eng.alloc_cols(N)
rows = {"rows": eng.alloc_rows(N)}
flush = torch.empty(512 << 20, dtype=torch.uint8, device="cuda")  # > Infinity Cache
for _ in range(3):
    flush.fill_(1)
    eng.stream_read(slab, grid=2048)
    for v in (0, 5, 3):
        flush.fill_(1)
        eng.set_unpack_variant(v)
        eng.unpack(slab, N, stride=REC, fixed_len=REC, cols=cols)
    eng.set_unpack_variant(0)
    flush.fill_(1)
    eng.unpack(slab, N, stride=REC, fixed_len=REC, cols=rows)
    flush.fill_(1)
    eng.unpack(slab, N, stride=REC, fixed_len=REC, cols=cols, opts=OPT_SKIP_CRC)
torch.cuda.synchronize()
assert int((cols["err"] != 0).sum()) == 0
print("traffic probe done")
