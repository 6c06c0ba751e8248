"""Phase stamps of the scan's chain kernel (diagnostics build): the config-5 stream scanned 20
times, then s_memtime stamps of the last call's groups 0..63 (start, counts prefix, marks, H
list, look-back, end), in shader clocks relative to each group's start (the counters of
different XCDs are not aligned)."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mgen_amd import PACK_CHECKSUM, SCAN_TCP, Engine, to_device  # noqa: E402
from mgen_amd._abi import DESC_DTYPE  # noqa: E402
from mgen_amd.workloads import make_templates  # noqa: E402

n = 65536
eng = Engine(0, diag=True)
tmpl, pool = make_templates(64)
desc = np.zeros(n, DESC_DTYPE)
seq = np.arange(n)
desc["tmpl"], desc["seq_num"] = seq % 64, seq
desc["tx_sec"], desc["tx_usec"], desc["flags"] = 1_700_000_000, seq % 1_000_000, 4
tm, pl = to_device(tmpl), to_device(pool)
tcrc = torch.empty(64, dtype=torch.int32, device="cuda")
eng.pack_prepare(tm, 64, pl, tcrc)
d_total = torch.full((n,), 16384, dtype=torch.int32, device="cuda")
local, _ = eng.pack_tcp(tm, tcrc, to_device(desc), d_total, n, pl, opts=PACK_CHECKSUM)
out = (torch.empty(n + 1, dtype=torch.int64, device="cuda"),
       torch.empty(n + 1, dtype=torch.int32, device="cuda"))
for _ in range(20):
    offs, lens, info = eng.stream_scan(local, SCAN_TCP, out=out)
torch.cuda.synchronize()
print("path", int(info.path), "records", int(info.n_records), flush=True)
st = np.zeros(512, np.uint64)
assert eng.lib.mgenx_diag_chain_prof(ctypes.c_void_p(st.ctypes.data)) == 0
st = st.reshape(64, 8).astype(np.int64)
rel = st[:, 1:6] - st[:, :1]
starts = st[:, 0] - st[:, 0].min()
names = ["prefix", "marks", "hlist", "lookback", "end"]
print("median clocks from group start:", dict(zip(names, np.median(rel, 0).tolist())))
print("max clocks from group start:", dict(zip(names, rel.max(0).tolist())))
eng.close()
