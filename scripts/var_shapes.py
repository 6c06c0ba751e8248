"""Config 3 unpack (1M records, U{64..1472}, back to back, checksummed, 32-B rows) through the
var-kernel shapes of the diagnostics build (MGENX_TUNE_UNPACK_VARIANT 20..29, see
launch_unpack): block size, rows held for burst stores, the store ablation, ticket-scheduled
tiles.  Every shape's rows are compared with the product kernel's (bit-exact) before timing.
Also 1M x 1024-B records given as offsets + lengths (the structural comparison of var_probe)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mgen_amd import PACK_CHECKSUM, Engine, to_device  # noqa: E402
from mgen_amd.workloads import udp_fixed, udp_mixed  # noqa: E402

N = 1 << 20
eng = Engine(0, diag=True)
rows = {"rows": eng.alloc_rows(N)}
VARIANTS = [int(v) for v in os.environ.get("VARIANTS", "0,20,21,22,23,24,25,26,27,28,29").split(",")]


def timed(fn, reps=20):
    fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def sweep(name, slab, d_of, d_len, total):
    """every variant checked against the product rows once, then timed ROUNDS times in
    interleaved order (A B C A B C ...): the first timings on a box run slow"""
    eng.set_unpack_variant(0)
    eng.unpack(slab, N, rec_off=d_of, rec_len=d_len, cols=rows)
    torch.cuda.synchronize()
    ref = rows["rows"].clone()
    for v in VARIANTS:
        eng.set_unpack_variant(v)
        rows["rows"].zero_()
        eng.unpack(slab, N, rec_off=d_of, rec_len=d_len, cols=rows)
        torch.cuda.synchronize()
        same = bool(torch.equal(rows["rows"], ref))
        print(f"{name} variant {v:3d}: rows {'== product' if same else 'DIFFER'} "
              f"kernel {eng.last_unpack_kernel()}", flush=True)
    res = {v: [] for v in VARIANTS}
    for _ in range(int(os.environ.get("ROUNDS", "5"))):
        for v in VARIANTS:
            eng.set_unpack_variant(v)
            res[v].append(timed(lambda: eng.unpack(slab, N, rec_off=d_of, rec_len=d_len, cols=rows)))
    for v in VARIANTS:
        t = sorted(res[v])
        print(f"{name} variant {v:3d}: median {t[len(t) // 2]:.4f} ms min {t[0]:.4f} "
              f"({total / 1e9 / t[len(t) // 2]:.2f} TB/s)  all {' '.join(f'{x:.4f}' for x in res[v])}",
              flush=True)
    eng.set_unpack_variant(0)


tm, pl, ds, of, sz = udp_mixed(N, 64, 1472, 64, payload_hex="00112233445566778899aabbccddeeff")
total = int(of[-1] + sz[-1])
dt, dp = to_device(tm), to_device(pl)
c = torch.empty(len(tm), dtype=torch.int32, device="cuda")
eng.pack_prepare(dt, len(tm), dp, c)
slab = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
d_of = to_device(of).view(torch.int64)
eng.pack(dt, c, to_device(ds), N, dp, slab, rec_off=d_of, opts=PACK_CHECKSUM)
d_len = to_device(sz).view(torch.int32)
sweep("config3", slab, d_of, d_len, total + 32 * N)
del slab

if os.environ.get("FIXED", "1") == "1":
    L = 1024
    t, p, d = udp_fixed(N, L)
    dt, dp = to_device(t), to_device(p)
    c = torch.empty(len(t), dtype=torch.int32, device="cuda")
    eng.pack_prepare(dt, len(t), dp, c)
    slab = torch.empty(N * L + 64, dtype=torch.uint8, device="cuda")
    eng.pack(dt, c, to_device(d), N, dp, slab, stride=L, opts=PACK_CHECKSUM)
    offs = torch.arange(N, dtype=torch.int64, device="cuda") * L
    lens = torch.full((N,), L, dtype=torch.int32, device="cuda")
    sweep("fixed1024", slab, offs, lens, N * (L + 32))
    eng.set_unpack_variant(0)
    ms_fix = timed(lambda: eng.unpack(slab, N, stride=L, fixed_len=L, cols=rows))
    print(f"fixed1024 ring kernel: {ms_fix:.4f} ms", flush=True)
