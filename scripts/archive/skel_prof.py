"""flow_skel_kernel phase cycles (diagnostics build): config-4 data, the full set and rank 0's
share at N = 8; the first walk to finish reports s_memtime cycles of its fast runs, prefix
scans, event records, total and staging (the records into LDS, incl. the wait), and counts."""
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
names = ["fast", "scans", "events", "total", "staging", "fast_n", "slow_n", "events_n"]
for name, sel in (("full", None), ("share8", 0)):
    dd = d if sel is None else {k: np.ascontiguousarray(v[(d["flow_id"] % 8) == sel])
                                for k, v in d.items()}
    t = {k: torch.from_numpy(v).cuda() for k, v in dd.items()}
    idx = torch.from_numpy((dd["flow_id"] - 1).astype(np.uint32)).cuda()
    buf = (ctypes.c_ulonglong * 8)()
    for _ in range(3):
        flows = eng.flow_init(1024, 1.0)
        eng.flow_reduce(flows, 1024, idx, t["seq"], t["tx_sec"], t["tx_usec"], t["msg_len"],
                        t["rx_sec"], t["rx_usec"], n=len(dd["seq"]))
        torch.cuda.synchronize()
        assert eng.lib.mgenx_diag_seg_prof(buf, 8) == 0
    a = list(buf)
    print(name, " ".join("%s=%d" % (k, v) for k, v in zip(names, a)), flush=True)
    if a[5]:
        print("   per fast run:", "%.0f" % (a[0] / a[5]), " per event: %.0f" % (a[2] / max(a[7], 1)))
    wbuf = (ctypes.c_ulonglong * 8)()
    assert eng.lib.mgenx_diag_seg_prof(wbuf, 12) == 0
    wn = ["setup", "insert", "dups", "counters", "sums", "tail", "total", "chunks"]
    print(name, "window k=1:", " ".join("%s=%d" % (k, v) for k, v in zip(wn, list(wbuf))), flush=True)
