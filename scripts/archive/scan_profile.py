"""Config 5 stream scan alone (1 GiB of 16-KiB TCP records, oracle-built 64 MiB tiled 16x),
a few repetitions -- run under rocprofv3 --kernel-trace --stats for the per-kernel split."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mgen_amd import SCAN_TCP, Engine, to_device  # noqa: E402
from mgen_amd._abi import DESC_DTYPE  # noqa: E402
from mgen_amd.workloads import make_templates  # noqa: E402
from oracle import oracle as O  # noqa: E402

eng = Engine(0)
n0 = 4096
tmpl, pool = make_templates(64)
desc = np.zeros(n0, DESC_DTYPE)
desc["tmpl"] = np.arange(n0) % 64
desc["seq_num"] = np.arange(n0) // 64
desc["tx_sec"] = 1_700_000_000
desc["tx_usec"] = np.arange(n0)
desc["msg_len"] = 16384
desc["flags"] = 4
s0 = np.asarray(O.tcp_tx_batch(tmpl, desc, np.full(n0, 16384, np.uint32), pool), np.uint8)
stream = to_device(s0).repeat(16)
n = n0 * 16
for _ in range(2):
    eng.stream_scan(stream, SCAN_TCP, cap=n + 1)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(5):
    offs, lens, info = eng.stream_scan(stream, SCAN_TCP, cap=n + 1)
torch.cuda.synchronize()
print("scan_ms", (time.perf_counter() - t0) / 5 * 1e3, "records", int(info.n_records),
      "candidates", int(info.candidates), "nt", os.environ.get("MGENX_SCAN_NT", "0"))
if len(sys.argv) > 1 and sys.argv[1] == "read":
    d = Engine(0, diag=True)
    for _ in range(2):
        d.stream_read(stream, grid=4096)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        d.stream_read(stream, grid=4096)
    torch.cuda.synchronize()
    print("stream_read_ms", (time.perf_counter() - t0) / 10 * 1e3)
