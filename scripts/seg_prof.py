"""flow_seg_kernel phase stamps (diagnostics build): config-4 data, the full set and rank 0's
share at N = 8; prints, per wave of workgroup 0's first pass, the cycles (s_memtime) from the
pass start to each phase boundary."""
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
names = ["start", "walk0", "walk1", "scat", "ringin", "ringout", "class", "aggin", "replay", "skel", "scan", "post"]
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
    W = 16
    buf = (ctypes.c_ulonglong * (W * 12))()
    assert eng.lib.mgenx_diag_seg_prof(buf, W * 12) == 0
    a = np.array(list(buf), dtype=np.int64).reshape(W, 12)
    t0 = a[:, 0].min()
    print(name, "cycles from the pass start, per wave:", " ".join(names))
    for w in range(W):
        print("  w%d" % w, " ".join("%7d" % (x - t0) for x in a[w]))
