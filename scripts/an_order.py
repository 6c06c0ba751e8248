"""Timing of mgenx_flow_reduce on config-4 data (diagnostics build): the ordering alone
(MGENX_AN_SABL=1) and the whole reduce, for the full 8M records / 1024 flows and rank 0's share
at N = 8; with an argument, also the ordering with tile-contiguous writes (MGENX_AN_SEQW=1:
wrong results, the cost of the scattered runs).  (Round 4's phase cuts of the one-tile-per-block order kernel, MGENX_AN_OCUT, went
with that kernel.)"""
import os
import subprocess
import sys
import time

import numpy as np

if len(sys.argv) == 1 or sys.argv[1] != "run":
    runs = [("order_only", dict(MGENX_AN_SABL="1")), ("reduce", {})]
    if len(sys.argv) > 1 or os.environ.get("AN_ORDER_SEQW"):
        runs.append(("order_only_seqw", dict(MGENX_AN_SABL="1", MGENX_AN_SEQW="1")))
    for name, extra in runs:
        env = dict(os.environ, **extra)
        r = subprocess.run([sys.executable, __file__, "run"], env=env, capture_output=True,
                           text=True, timeout=300)
        print(name, r.stdout.strip()[-300:], r.stderr.strip()[-400:] if r.returncode else "",
              flush=True)
    sys.exit(0)

import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mgen_amd import Engine  # noqa: E402
from mgen_amd.workloads import poisson_flows  # noqa: E402

eng = Engine(0, diag=True)
d = poisson_flows(8388608, 1024, mean_gap_us=1000)
out = {}
for name, sel in (("full", None), ("share8", 0)):
    dd = d if sel is None else {k: np.ascontiguousarray(v[(d["flow_id"] % 8) == sel])
                                for k, v in d.items()}
    t = {k: torch.from_numpy(v).cuda() for k, v in dd.items()}
    idx = torch.from_numpy((dd["flow_id"] - 1).astype(np.uint32)).cuda()
    n = len(dd["seq"])

    def run():
        flows = eng.flow_init(1024, 1.0)
        eng.flow_reduce(flows, 1024, idx, t["seq"], t["tx_sec"], t["tx_usec"], t["msg_len"],
                        t["rx_sec"], t["rx_usec"], n=n)

    run()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        run()
    torch.cuda.synchronize()
    out[name] = round((time.perf_counter() - t0) / 10 * 1e3, 4)
print(out)
