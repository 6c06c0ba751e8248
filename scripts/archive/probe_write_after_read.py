"""Probe: cost of writing the 32 MB of output rows right after a 1 GiB read pass (the read
evicts the rows from the Infinity Cache), against the same write with the rows resident.
Events around each kernel; median of 10 alternations."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mgen_amd import Engine  # noqa: E402

eng = Engine(0, diag=True)
slab = torch.ones(1 << 30, dtype=torch.uint8, device="cuda")
rows = torch.empty(32 << 20, dtype=torch.uint8, device="cuda")
ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
res = {"read_only": [], "write_after_read": [], "write_resident": [], "read_after_write": [],
       "write_after_read_nt": []}
for _ in range(12):
    a, b, c, d, e, f = ev(), ev(), ev(), ev(), ev(), ev()
    a.record(); eng.group_rw(slab, rows, 0); b.record()
    rows.fill_(3); c.record()
    rows.fill_(4); d.record()
    eng.group_rw(slab, rows, 0); e.record()
    torch.cuda.synchronize()
    res["read_only"].append(a.elapsed_time(b))
    res["write_after_read"].append(b.elapsed_time(c))
    res["write_resident"].append(c.elapsed_time(d))
    res["read_after_write"].append(d.elapsed_time(e))
out = {k: round(float(np.median(v[2:])) * 1e3, 2) for k, v in res.items() if v}
print(json.dumps({"us": out}))
