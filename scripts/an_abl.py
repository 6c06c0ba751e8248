"""Timing of mgenx_flow_reduce on config 4 data with the diagnostics build's update-kernel
ablations (MGENX_AN_ABL bits: 1 no latency sum loop, 2 no general update, 4 no fast runs,
8 no run commit; "r" = abl 0 with the radix-sort ordering, MGENX_AN_RADIX; ordering only,
"s" = the ordering alone, MGENX_AN_SABL).  Results are wrong
under ablation; timing only."""
import os
import subprocess
import sys
import time

import numpy as np

if len(sys.argv) == 1:
    for a in os.environ.get("ABLS", "0,r,1,2,8,3,4").split(","):
        env = dict(os.environ, MGENX_AN_ABL="0" if a in "rs" else a,
                   MGENX_AN_RADIX="1" if a == "r" else "0",
                   MGENX_AN_SABL="1" if a == "s" else "0")
        r = subprocess.run([sys.executable, __file__, "run"], env=env, capture_output=True,
                           text=True, timeout=200)
        print("abl", a, r.stdout.strip()[-200:], r.stderr.strip()[-300:] if r.returncode else "")
    sys.exit(0)

import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mgen_amd import Engine  # noqa: E402
from mgen_amd.workloads import poisson_flows  # noqa: E402

eng = Engine(0, diag=True)
d = poisson_flows(8388608, 1024, mean_gap_us=1000)
if os.environ.get("SORTED") == "1":   # input already in flow order: `order` is the identity
    o = np.argsort(d["flow_id"], kind="stable")
    d = {k: np.ascontiguousarray(v[o]) for k, v in d.items()}
t = {k: torch.from_numpy(v).cuda() for k, v in d.items()}
idx = torch.from_numpy((d["flow_id"] - 1).astype(np.uint32)).cuda()
n = len(d["seq"])


def run():
    flows = eng.flow_init(1024, 1.0)
    eng.flow_reduce(flows, 1024, idx, t["seq"], t["tx_sec"], t["tx_usec"], t["msg_len"],
                    t["rx_sec"], t["rx_usec"], n=n)


run()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(5):
    run()
torch.cuda.synchronize()
print("reduce_ms", round((time.perf_counter() - t0) / 5 * 1e3, 4))
