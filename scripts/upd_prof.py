"""flow_update_kernel and flow_order_kernel phase cycles (diagnostics build): config-4 data, the full set and rank 0's
share at N = 8; prints the s_memtime cycles workgroup 0's first wave spent per phase (event
detection incl. load waits, bulk runs, exact steps, lat' store + tail) and the counts."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mgen_amd import Engine  # noqa: E402
from mgen_amd.workloads import poisson_flows  # noqa: E402

eng = Engine(0, diag=True)
d = poisson_flows(8388608, 1024, mean_gap_us=1000)
names = ["detect", "bulk", "exact_other", "store", "rounds", "exact_n", "bulk_n", "total",
         "restart", "restart_n"]
for name, sel in (("full", None), ("share8", 0)):
    dd = d if sel is None else {k: np.ascontiguousarray(v[(d["flow_id"] % 8) == sel])
                                for k, v in d.items()}
    t = {k: torch.from_numpy(v).cuda() for k, v in dd.items()}
    idx = torch.from_numpy((dd["flow_id"] - 1).astype(np.uint32)).cuda()
    for _ in range(3):
        flows = eng.flow_init(1024, 1.0)
        eng.flow_reduce(flows, 1024, idx, t["seq"], t["tx_sec"], t["tx_usec"], t["msg_len"],
                        t["rx_sec"], t["rx_usec"], n=len(dd["seq"]))
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * 10)()
    assert eng.lib.mgenx_diag_seg_prof(buf, 10) == 0
    a = list(buf)
    print(name, " ".join("%s=%d" % (k, v) for k, v in zip(names, a)))
    if a[4]:
        print("   per round:", " ".join("%s=%.0f" % (k, v / a[4]) for k, v in zip(names[:4], a[:4])))
    buf = (ctypes.c_ulonglong * 16)()
    assert eng.lib.mgenx_diag_seg_prof(buf, 16) == 0
    b = list(buf)[:8]
    onames = ["count", "scan", "rank_place", "prefetch", "write", "tiles", "-", "total"]
    print(name, "order:", " ".join("%s=%d" % (k, v) for k, v in zip(onames, b)))
    if b[5]:
        print("   per tile:", " ".join("%s=%.0f" % (k, v / b[5]) for k, v in zip(onames[:5], b[:5])))
