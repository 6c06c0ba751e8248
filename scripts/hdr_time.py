"""Header-only decode timings: config 2's 1M x 1024-B slab with MGENX_OPT_SKIP_CRC (the
general kernel's header-only path) and config 4's 8.4M x 256-B datagrams without the
CHECKSUM flag into rows (the fixed kernel's header-only mode)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from mgen_amd import DESC_DTYPE, OPT_SKIP_CRC, Engine, to_device  # noqa: E402
from mgen_amd.workloads import make_templates  # noqa: E402

eng = Engine(0)
dev = torch.device("cuda:0")
from mgen_amd import PACK_CHECKSUM  # noqa: E402
from mgen_amd.workloads import udp_fixed  # noqa: E402
tmpl, pool, desc = udp_fixed(bench.N_REC, bench.REC)
d_tmpl, d_pool, d_desc = (to_device(a, eng.device) for a in (tmpl, pool, desc))
tcrc = torch.empty(len(tmpl), dtype=torch.int32, device=dev)
eng.pack_prepare(d_tmpl, len(tmpl), d_pool, tcrc)
slab = torch.empty(bench.N_REC * bench.REC, dtype=torch.uint8, device=dev)
eng.pack(d_tmpl, tcrc, d_desc, bench.N_REC, d_pool, slab, stride=bench.REC, opts=PACK_CHECKSUM)
if True:
    cols = eng.alloc_cols(bench.N_REC)
    ms = bench.timed(torch, lambda: eng.unpack(slab, bench.N_REC, stride=bench.REC, fixed_len=bench.REC,
                                               opts=OPT_SKIP_CRC, cols=cols), reps=20)
    print(f"config2 header-only ms {ms:.4f}")
n, n_flows, msg = bench.N4_TOTAL, 1024, 256
tmpl, pool = make_templates(n_flows)
desc = np.zeros(n, DESC_DTYPE)
desc["tmpl"], desc["seq_num"] = np.arange(n) % n_flows, np.arange(n) // n_flows
desc["tx_sec"], desc["tx_usec"], desc["msg_len"] = 1_700_000_000, np.arange(n) % 1_000_000, msg
dt, dp = to_device(tmpl, eng.device), to_device(pool, eng.device)
crc = torch.empty(n_flows, dtype=torch.int32, device=dev)
eng.pack_prepare(dt, n_flows, dp, crc)
s4 = torch.empty(n * msg, dtype=torch.uint8, device=dev)
eng.pack(dt, crc, to_device(desc, eng.device), n, dp, s4, stride=msg)
rows = {"rows": eng.alloc_rows(n)}
ms = bench.timed(torch, lambda: eng.unpack(s4, n, stride=msg, fixed_len=msg, cols=rows), reps=10)
print(f"config4 rows unpack ms {ms:.4f}  (kernel {eng.last_unpack_kernel()})")
