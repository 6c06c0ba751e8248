"""Ablation timing for the CRC unpack kernel on the config-2 batch (interleaved rounds in
one process, cdna_hip_programming.md 5.4 rule 24): mode 0 = product kernel, 1 = loads+XOR
(no LDS lookups), 2 = lookups on L1-resident rows (no streaming), header-only, and a plain
streaming read of the same slab at several grid sizes."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mgen_amd import OPT_SKIP_CRC, PACK_CHECKSUM, Engine, to_device  # noqa: E402
from mgen_amd.workloads import udp_fixed  # noqa: E402

N, REC = 1 << 20, 1024
ALGO = N * REC + N * 32
eng = Engine(0, diag=True)
tmpl, pool, desc = udp_fixed(N, REC)
d_tmpl, d_pool, d_desc = to_device(tmpl), to_device(pool), to_device(desc)
crc = torch.empty(len(tmpl), dtype=torch.int32, device="cuda")
eng.pack_prepare(d_tmpl, len(tmpl), d_pool, crc)
slab = torch.empty(N * REC, dtype=torch.uint8, device="cuda")
eng.pack(d_tmpl, crc, d_desc, N, d_pool, slab, stride=REC, opts=PACK_CHECKSUM)
cols = eng.alloc_cols(N)
rows = {"rows": eng.alloc_rows(N)}
eng.set_unpack_variant(0)
eng.unpack(slab, N, stride=REC, fixed_len=REC, cols=cols)
torch.cuda.synchronize()
assert int((cols["err"] != 0).sum()) == 0


def run(name):
    """c<V> / r<V>: columns / 32-B rows with unpack variant V; hdr_*: checksum off;
    read_<G>: plain streaming read of the slab with grid G."""
    if name[0] in "cr" and name[1:].isdigit():
        eng.set_unpack_variant(int(name[1:]))
        eng.unpack(slab, N, stride=REC, fixed_len=REC, cols=cols if name[0] == "c" else rows)
    elif name == "hdr_rows":
        eng.set_unpack_variant(0)
        eng.unpack(slab, N, stride=REC, fixed_len=REC, cols=rows, opts=OPT_SKIP_CRC)
    elif name == "hdr_only":
        eng.set_unpack_variant(0)
        eng.unpack(slab, N, stride=REC, fixed_len=REC, cols=cols, opts=OPT_SKIP_CRC)
    elif name.startswith("grw"):  # grw<mode>: group read (+ row stores)
        eng.group_rw(slab, rows["rows"], int(name[3:]))
    elif name == "fill_rows":
        rows["rows"].fill_(1)
    else:
        eng.stream_read(slab, grid=int(name.split("_")[1]))


names = os.environ.get("SWEEP_NAMES", "").split(",") if os.environ.get("SWEEP_NAMES") else [
    "c0", "r0", "c12", "c33", "c34", "c35", "c36", "c37", "c40", "c48", "r48", "hdr_only",
    "read_8192"]
res = {k: [] for k in names}
for rnd in range(7):
    for k in names:
        run(k)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(10):
            run(k)
        b.record()
        torch.cuda.synchronize()
        res[k].append(a.elapsed_time(b) / 10)
eng.set_unpack_variant(0)
out = {}
for k, t in res.items():
    ms = float(np.median(t))
    byts = N * REC if k.startswith("read") else (N * 32 if k == "fill_rows" else ALGO)
    out[k] = {"ms": round(ms, 4), "GBps": round(byts / ms / 1e6, 1)}
print(json.dumps(out))
