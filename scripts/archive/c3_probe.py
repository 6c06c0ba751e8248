"""Config-3 diagnostics: general-kernel pack/unpack on mixed sizes, the same sizes sorted
(globally / within 1024-record tiles) and one uniform size, to size the padding loss."""
import json
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from bench import timed  # noqa: E402
from mgen_amd import PACK_CHECKSUM, Engine, to_device  # noqa: E402
from mgen_amd.workloads import udp_mixed  # noqa: E402


def run(eng, name, sizes_fn):
    n = 1 << 20
    tmpl, pool, desc, offs, sizes = udp_mixed(n, 64, 1472, 64,
                                              payload_hex="00112233445566778899aabbccddeeff")
    sizes = sizes_fn(sizes.astype(np.int64))
    desc["msg_len"] = sizes.astype(np.uint16)
    offs = np.zeros(n, np.uint64)
    offs[1:] = np.cumsum(sizes[:-1])
    total = int(offs[-1] + sizes[-1])
    dev = "cuda:0"
    d_tmpl, d_pool, d_desc = to_device(tmpl), to_device(pool), to_device(desc)
    d_offs = to_device(offs).view(torch.int64)
    d_len = to_device(sizes.astype(np.uint32)).view(torch.int32)
    crc = torch.empty(len(tmpl), dtype=torch.int32, device=dev)
    eng.pack_prepare(d_tmpl, len(tmpl), d_pool, crc)
    slab = torch.empty(total + 64, dtype=torch.uint8, device=dev)
    out_len = torch.empty(n, dtype=torch.int32, device=dev)
    cols = eng.alloc_cols(n)
    pack = lambda: eng.pack(d_tmpl, crc, d_desc, n, d_pool, slab, rec_off=d_offs,  # noqa
                            opts=PACK_CHECKSUM, out_len=out_len)
    unpack = lambda: eng.unpack(slab, n, rec_off=d_offs, rec_len=d_len, cols=cols)  # noqa
    pms, ums = timed(torch, pack), timed(torch, unpack)
    assert var in (1, 2) or pvar or int((cols["err"] != 0).sum()) == 0
    pb, ub = n * 36 + total, total + n * 32
    print(json.dumps({"case": name, "bytes": total, "pack_ms": round(pms, 4),
                      "unpack_ms": round(ums, 4), "pack_gbps": round(pb / pms / 1e6),
                      "unpack_gbps": round(ub / ums / 1e6),
                      "combined": round((pb + ub) / (pms + ums) / 1e6)}), flush=True)


def tile_sort(s, t=1024):
    s = s.copy()
    for a in range(0, len(s), t):
        s[a:a + t] = np.sort(s[a:a + t])
    return s


CASES = {
    "mixed": lambda s: s,
    "sorted": np.sort,
    "tile_sorted_1024": tile_sort,
    "tile_sorted_256": lambda s: tile_sort(s, 256),
    "uniform_768": lambda s: np.full_like(s, 768),
    "uniform_769": lambda s: np.full_like(s, 769),
    "uniform_772": lambda s: np.full_like(s, 772),
    "uniform_1472": lambda s: np.full_like(s, 1472),
    "mixed_x16": lambda s: (s + 15) // 16 * 16,
}
var = int(sys.argv[2]) if len(sys.argv) > 2 else 0
pvar = int(sys.argv[3]) if len(sys.argv) > 3 else 0   # pack ablation (diag build)
# argv[1]: cases; argv[2] (optional): unpack variant on the diagnostics build (3 = unsorted)
eng = Engine(0, diag=var != 0 or pvar != 0)
if var:
    assert eng.lib.mgenx_set_tuning(eng.ctx, 1, var) == 0
if pvar:
    assert eng.lib.mgenx_set_tuning(eng.ctx, 2, pvar) == 0
for name in (sys.argv[1].split(",") if len(sys.argv) > 1 else CASES):
    run(eng, name + ("" if not var else f"/v{var}") + ("" if not pvar else f"/p{pvar}"), CASES[name])
eng.close()
