"""TCP transmit timing: config 5's stream (65,536 x 16 KiB, checksum on) built by
mgenx_pack_tcp, 20 calls after one warm call (bench.py's tcp_tx leg alone)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mgen_amd import PACK_CHECKSUM, Engine, to_device  # noqa: E402
from mgen_amd._abi import DESC_DTYPE  # noqa: E402
from mgen_amd.workloads import make_templates  # noqa: E402

n = 65536
# python scripts/tcp_time.py [V]: with V, the diagnostics build at pack variant V
eng = Engine(0, diag=len(sys.argv) > 1)
if len(sys.argv) > 1:
    eng.set_pack_variant(int(sys.argv[1]))
tmpl, pool = make_templates(64)
desc = np.zeros(n, DESC_DTYPE)
seq = np.arange(n)
desc["tmpl"], desc["seq_num"] = seq % 64, seq
desc["tx_sec"], desc["tx_usec"], desc["flags"] = 1_700_000_000, seq % 1_000_000, 4
tm, pl = to_device(tmpl), to_device(pool)
tcrc = torch.empty(64, dtype=torch.int32, device="cuda")
eng.pack_prepare(tm, 64, pl, tcrc)
d_desc = to_device(desc)
d_total = torch.full((n,), 16384, dtype=torch.int32, device="cuda")
local, offs = eng.pack_tcp(tm, tcrc, d_desc, d_total, n, pl, opts=PACK_CHECKSUM)
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
for _ in range(20):
    eng.pack_tcp(tm, tcrc, d_desc, d_total, n, pl, opts=PACK_CHECKSUM, out=local, offs=offs)
b.record()
torch.cuda.synchronize()
print("tcp_tx_ms", a.elapsed_time(b) / 20, flush=True)
