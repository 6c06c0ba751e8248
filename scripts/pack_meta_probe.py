"""Is config 2's pack bound by its meta phase?  The same pack with and without the checksum
(the checksum is most of phase 1's work: the header CRC through LDS tables and the CRC
algebra) and with the diagnostics variant 2 (CRC skipped inside the kernel)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mgen_amd import PACK_CHECKSUM, Engine, to_device  # noqa: E402
from mgen_amd.workloads import udp_fixed  # noqa: E402


def timed(fn, reps=30):
    fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


n = 1 << 20
d = Engine(0, diag=True)
tmpl, pool, desc = udp_fixed(n, 1024)
dt, dp, dd = to_device(tmpl), to_device(pool), to_device(desc)
crc = torch.empty(len(tmpl), dtype=torch.int32, device="cuda")
d.pack_prepare(dt, len(tmpl), dp, crc)
slab = torch.empty(n * 1024, dtype=torch.uint8, device="cuda")
ol = torch.empty(n, dtype=torch.int32, device="cuda")
for rnd in range(3):
    for v, opts, name in ((0, PACK_CHECKSUM, "checksum"), (0, 0, "no checksum"),
                          (2, PACK_CHECKSUM, "variant 2 (CRC skipped)")):
        d.set_pack_variant(v)
        ms = timed(lambda: d.pack(dt, crc, dd, n, dp, slab, stride=1024, opts=opts, out_len=ol))
        print(f"round {rnd} {name}: {ms:.4f} ms")
d.set_pack_variant(0)
