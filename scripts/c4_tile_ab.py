"""A/B in one process (diagnostics build): config 4's reduce and rank 0's share at N = 8, with
the order kernel's tile size forced (MGENX_AN_TILE = 4096 / 4608, read per call) and with or
without a report-count array (the caller's zero fill that per_flow = 0 no longer needs),
interleaved over three rounds."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from mgen_amd import Engine  # noqa: E402
from mgen_amd.workloads import poisson_flows  # noqa: E402

eng = Engine(0, diag=True)
d = poisson_flows(bench.N4_TOTAL, 1024, mean_gap_us=1000)
sets = {}
for name, sel in (("full", None), ("share8", 0)):
    dd = d if sel is None else {k: np.ascontiguousarray(v[(d["flow_id"] % 8) == sel])
                                for k, v in d.items()}
    t = {k: torch.from_numpy(v).cuda() for k, v in dd.items()}
    t["idx"] = torch.from_numpy((dd["flow_id"] - 1).astype(np.uint32)).cuda()
    sets[name] = (t, len(dd["seq"]))


def run(t, n, with_count):
    flows = eng.flow_init(1024, 1.0)
    rc = torch.zeros(1024, dtype=torch.int32, device="cuda") if with_count else None
    eng.flow_reduce(flows, 1024, t["idx"], t["seq"], t["tx_sec"], t["tx_usec"], t["msg_len"],
                    t["rx_sec"], t["rx_usec"], n=n, report_count=rc)


out = {}
for rnd in range(3):
    for name, (t, n) in sets.items():
        for tile in ("4096", "4608"):
            for wc in (True, False):
                os.environ["MGENX_AN_TILE"] = tile
                key = f"{name}/tile{tile}/{'count' if wc else 'nocount'}"
                out.setdefault(key, []).append(round(bench.timed(torch, lambda: run(t, n, wc)), 4))
print(json.dumps(out))
