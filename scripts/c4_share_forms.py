"""Rank 0's share of config 4 at N = 8 (flows with flow_id mod 8 == 0: 128 flows, 1/8 of the
records), timed two ways on one GPU: the flow states numbered globally (1024 slots, 7/8 of them
idle on this rank) and rank-locally (128 slots: global index g -> g // 8).  Both runs are
checked against each other (every state of the local run equals the global run's state of
the same flow)."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from mgen_amd import FLOW_STATE_BYTES, Engine  # noqa: E402
from mgen_amd.workloads import poisson_flows  # noqa: E402

eng = Engine(0)
d = poisson_flows(bench.N4_TOTAL, 1024, mean_gap_us=1000)
own = (d["flow_id"] % 8) == 0
d = {k: np.ascontiguousarray(v[own]) for k, v in d.items()}
n = len(d["seq"])
g = (d["flow_id"] - 1).astype(np.uint32)
t = {k: torch.from_numpy(v).cuda() for k, v in d.items()}
out = {"records": n}
states = {}
for name, idx, nf in (("global_1024", g, 1024), ("local_128", g // 8, 128)):
    ti = torch.from_numpy(idx).cuda()

    def run():
        f = eng.flow_init(nf, 1.0)
        states[name] = f
        eng.flow_reduce(f, nf, ti, t["seq"], t["tx_sec"], t["tx_usec"], t["msg_len"],
                        t["rx_sec"], t["rx_usec"], n=n)
    ms = [bench.timed(torch, run, reps=10) for _ in range(3)]
    out[name] = [round(x, 4) for x in ms]
gl = states["global_1024"].cpu().numpy().reshape(1024, FLOW_STATE_BYTES)
lo = states["local_128"].cpu().numpy().reshape(128, FLOW_STATE_BYTES)
assert np.array_equal(gl[np.arange(128) * 8 + 7], lo), "local numbering changed a flow state"
out["checked"] = "local states == global states of the same flows"
print(json.dumps(out))
