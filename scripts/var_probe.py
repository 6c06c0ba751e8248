"""unpack_var_kernel on fixed-size records given as offsets + lengths (1M records of 1024,
768 and 769 B, back to back, checksummed) beside the fixed-stride kernels on the same slab,
and config 3: where the variable-length kernel loses against the fixed one."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mgen_amd import PACK_CHECKSUM, Engine, to_device  # noqa: E402
from mgen_amd.workloads import udp_fixed, udp_mixed  # noqa: E402

N = 1 << 20
eng = Engine(0)
rows = {"rows": eng.alloc_rows(N)}


def timed(fn, reps=20):
    fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


for L in (1024, 768, 769):
    t, p, d = udp_fixed(N, L)
    dt, dp = to_device(t), to_device(p)
    c = torch.empty(len(t), dtype=torch.int32, device="cuda")
    eng.pack_prepare(dt, len(t), dp, c)
    slab = torch.empty(N * L + 64, dtype=torch.uint8, device="cuda")
    eng.pack(dt, c, to_device(d), N, dp, slab, stride=L, opts=PACK_CHECKSUM)
    offs = torch.arange(N, dtype=torch.int64, device="cuda") * L
    lens = torch.full((N,), L, dtype=torch.int32, device="cuda")
    ms_var = timed(lambda: eng.unpack(slab, N, rec_off=offs, rec_len=lens, cols=rows))
    assert eng.last_unpack_kernel() == 3, eng.last_unpack_kernel()
    err = (rows["rows"].view(torch.int32).view(N, 8)[:, 6] >> 24) & 0xFF
    assert int((err != 0).sum()) == 0
    ms_fix = timed(lambda: eng.unpack(slab, N, stride=L, fixed_len=L, cols=rows))
    gb = N * L / 1e9
    print(f"L={L}: var {ms_var:.4f} ms ({gb / ms_var:.2f} TB/s)  fixed {ms_fix:.4f} ms "
          f"({gb / ms_fix:.2f} TB/s)", flush=True)
    del slab
tm, pl, ds, of, sz = udp_mixed(N, 64, 1472, 64, payload_hex="00112233445566778899aabbccddeeff")
total = int(of[-1] + sz[-1])
dt, dp = to_device(tm), to_device(pl)
c = torch.empty(len(tm), dtype=torch.int32, device="cuda")
eng.pack_prepare(dt, len(tm), dp, c)
slab = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
d_of = to_device(of).view(torch.int64)
eng.pack(dt, c, to_device(ds), N, dp, slab, rec_off=d_of, opts=PACK_CHECKSUM)
d_len = to_device(sz).view(torch.int32)
ms = timed(lambda: eng.unpack(slab, N, rec_off=d_of, rec_len=d_len, cols=rows))
print(f"config 3: var {ms:.4f} ms ({total / 1e9 / ms:.2f} TB/s)", flush=True)
