"""Pack timings: config 2 (1M x 1024 B, stride) and config 3 (1M x U{64..1472}, packed)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mgen_amd import PACK_CHECKSUM, Engine, to_device  # noqa: E402
from mgen_amd.workloads import udp_fixed, udp_mixed  # noqa: E402

eng = Engine(0)
dev = "cuda:0"


def timed(fn, reps=20):
    fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


n = 1 << 20
tmpl, pool, desc = udp_fixed(n, 1024)
dt, dp, dd = to_device(tmpl), to_device(pool), to_device(desc)
crc = torch.empty(len(tmpl), dtype=torch.int32, device=dev)
eng.pack_prepare(dt, len(tmpl), dp, crc)
slab = torch.empty(n * 1024, dtype=torch.uint8, device=dev)
ol = torch.empty(n, dtype=torch.int32, device=dev)
ms = timed(lambda: eng.pack(dt, crc, dd, n, dp, slab, stride=1024, opts=PACK_CHECKSUM, out_len=ol))
print(f"config2 pack_ms {ms:.4f} GB/s {(n * 1044) / ms / 1e6:.1f}")
tmpl, pool, desc, offs, sizes = udp_mixed(n, 64, 1472, 64, payload_hex="00112233445566778899aabbccddeeff")
total = int(offs[-1] + sizes[-1])
dt, dp, dd = to_device(tmpl), to_device(pool), to_device(desc)
do = to_device(offs).view(torch.int64)
crc = torch.empty(len(tmpl), dtype=torch.int32, device=dev)
eng.pack_prepare(dt, len(tmpl), dp, crc)
slab = torch.empty(total + 64, dtype=torch.uint8, device=dev)
ms = timed(lambda: eng.pack(dt, crc, dd, n, dp, slab, rec_off=do, opts=PACK_CHECKSUM, out_len=ol))
print(f"config3 pack_ms {ms:.4f} GB/s {(n * 36 + total) / ms / 1e6:.1f}")
if len(sys.argv) > 1:
    d = Engine(0, diag=True)
    for v in [0, 1, 3, 4, 5, 6, 7, 8, 9]:
        d.set_pack_variant(v)
        tmpl, pool, desc = udp_fixed(n, 1024)
        dt, dp, dd = to_device(tmpl), to_device(pool), to_device(desc)
        crc = torch.empty(len(tmpl), dtype=torch.int32, device=dev)
        d.pack_prepare(dt, len(tmpl), dp, crc)
        slab2 = torch.empty(n * 1024, dtype=torch.uint8, device=dev)
        ms = timed(lambda: d.pack(dt, crc, dd, n, dp, slab2, stride=1024, opts=PACK_CHECKSUM, out_len=ol))
        print(f"variant {v} config2 pack_ms {ms:.4f}")
if len(sys.argv) > 1:
    tmpl, pool, desc, offs, sizes = udp_mixed(n, 64, 1472, 64, payload_hex="00112233445566778899aabbccddeeff")
    total = int(offs[-1] + sizes[-1])
    dt, dp, dd = to_device(tmpl), to_device(pool), to_device(desc)
    do = to_device(offs).view(torch.int64)
    crc = torch.empty(len(tmpl), dtype=torch.int32, device=dev)
    d.pack_prepare(dt, len(tmpl), dp, crc)
    slab3 = torch.empty(total + 64, dtype=torch.uint8, device=dev)
    for v in [0, 1, 3, 4, 5, 6, 7, 8, 9]:
        d.set_pack_variant(v)
        ms = timed(lambda: d.pack(dt, crc, dd, n, dp, slab3, rec_off=do, opts=PACK_CHECKSUM, out_len=ol))
        print(f"variant {v} config3 pack_ms {ms:.4f}")
if len(sys.argv) > 1:
    # config 3 unpack: columns vs 32-B rows
    d.set_pack_variant(0)
    dl = to_device(sizes).view(torch.int32)
    d.pack(dt, crc, dd, n, dp, slab3, rec_off=do, opts=PACK_CHECKSUM, out_len=ol)
    cols = d.alloc_cols(n)
    ms = timed(lambda: d.unpack(slab3, n, rec_off=do, rec_len=dl, cols=cols))
    print(f"config3 unpack cols_ms {ms:.4f}")
    rc = {"rows": d.alloc_rows(n)}
    ms = timed(lambda: d.unpack(slab3, n, rec_off=do, rec_len=dl, cols=rc))
    print(f"config3 unpack rows_ms {ms:.4f}")
    assert int(((rc["rows"].view(torch.int32).view(n, 8)[:, 6] >> 24) & 0xFF).sum()) == 0
if len(sys.argv) > 1:
    # the same records at 16-byte-aligned starts (gaps of < 16 B): misalignment cost
    sz = sizes.astype(np.int64)
    al = (sz + 15) & ~15
    offs_al = np.zeros(n, np.uint64)
    offs_al[1:] = np.cumsum(al[:-1])
    tot_al = int(offs_al[-1] + al[-1]) + 64
    slab_al = torch.zeros(tot_al, dtype=torch.uint8, device=dev)
    do_al = to_device(offs_al).view(torch.int64)
    d.pack(dt, crc, dd, n, dp, slab_al, rec_off=do_al, opts=PACK_CHECKSUM, out_len=ol)
    rc2 = {"rows": d.alloc_rows(n)}
    ms = timed(lambda: d.unpack(slab_al, n, rec_off=do_al, rec_len=dl, cols=rc2))
    print(f"config3 aligned-starts unpack rows_ms {ms:.4f}")
    assert int(((rc2["rows"].view(torch.int32).view(n, 8)[:, 6] >> 24) & 0xFF).sum()) == 0
    # 64-byte-aligned starts
    al = (sz + 63) & ~63
    offs_al = np.zeros(n, np.uint64)
    offs_al[1:] = np.cumsum(al[:-1])
    tot_al = int(offs_al[-1] + al[-1]) + 64
    slab_al = torch.zeros(tot_al, dtype=torch.uint8, device=dev)
    do_al = to_device(offs_al).view(torch.int64)
    d.pack(dt, crc, dd, n, dp, slab_al, rec_off=do_al, opts=PACK_CHECKSUM, out_len=ol)
    ms = timed(lambda: d.unpack(slab_al, n, rec_off=do_al, rec_len=dl, cols=rc2))
    print(f"config3 64B-aligned-starts unpack rows_ms {ms:.4f}")
    # lengths rounded to multiples of 64 (rows exact), aligned
    sz64 = np.minimum(al, 1472)
    dl64 = to_device(sz64.astype(np.int32)).view(torch.int32)
    ms = timed(lambda: d.unpack(slab_al, n, rec_off=do_al, rec_len=dl64, cols=rc2))
    print(f"config3 64B-aligned, len%64==0 unpack rows_ms {ms:.4f} (CRC errors expected)")
if len(sys.argv) > 1:
    # record ENDS on the 16-byte grid (rows are aligned to the record end): row loads aligned
    ends = np.zeros(n, np.int64)
    offs_e = np.zeros(n, np.uint64)
    pe = 0
    for_i = np.arange(n)
    e = np.cumsum((sz + 15) & ~15)          # end_i = 16-aligned running end
    offs_e = (e - sz).astype(np.uint64)
    tot_e = int(e[-1]) + 64
    slab_e = torch.zeros(tot_e, dtype=torch.uint8, device=dev)
    do_e = to_device(offs_e).view(torch.int64)
    d.pack(dt, crc, dd, n, dp, slab_e, rec_off=do_e, opts=PACK_CHECKSUM, out_len=ol)
    ms = timed(lambda: d.unpack(slab_e, n, rec_off=do_e, rec_len=dl, cols=rc2))
    print(f"config3 end-aligned unpack rows_ms {ms:.4f}")
    assert int(((rc2["rows"].view(torch.int32).view(n, 8)[:, 6] >> 24) & 0xFF).sum()) == 0
