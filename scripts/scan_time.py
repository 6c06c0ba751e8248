"""Timing: whole-stream scan of bench.py's config-5 stream (GPU TCP transmit, 65,536 x
16 KiB records), 20 calls after one warm call; run under rocprofv3 --kernel-trace --stats
to count launches per call."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mgen_amd import PACK_CHECKSUM, PACK_RANDOM_FILL, SCAN_TCP, Engine, to_device  # noqa: E402
from mgen_amd._abi import DESC_DTYPE  # noqa: E402
from mgen_amd.workloads import make_templates  # noqa: E402

n = 65536
# DIAG=1: the diagnostics build (its env knobs, e.g. MGENX_SCAN_PLAIN); RF=1: RANDOM_FILL
# payloads (plausible record starts inside payloads: the lifting path)
eng = Engine(0, diag=os.environ.get("DIAG") == "1")
rf = os.environ.get("RF") == "1"
tmpl, pool = make_templates(64)
desc = np.zeros(n, DESC_DTYPE)
seq = np.arange(n)
desc["tmpl"] = seq % 64
desc["seq_num"] = seq
desc["tx_sec"] = 1_700_000_000
desc["tx_usec"] = seq % 1_000_000
desc["flags"] = 4
tm, pl = to_device(tmpl), to_device(pool)
tcrc = torch.empty(64, dtype=torch.int32, device="cuda")
eng.pack_prepare(tm, 64, pl, tcrc)
d_total = torch.full((n,), 16384, dtype=torch.int32, device="cuda")
local, _ = eng.pack_tcp(tm, tcrc, to_device(desc), d_total, n, pl, opts=PACK_CHECKSUM | (PACK_RANDOM_FILL if rf else 0))
out = (torch.empty(n + 1, dtype=torch.int64, device="cuda"),
       torch.empty(n + 1, dtype=torch.int32, device="cuda"))
offs, lens, info = eng.stream_scan(local, SCAN_TCP, out=out)
print("warm", int(info.n_records), int(info.candidates), int(info.resolved), flush=True)
torch.cuda.synchronize()
reps = 20
t0 = time.perf_counter()
for _ in range(reps):
    offs, lens, info = eng.stream_scan(local, SCAN_TCP, out=out)
torch.cuda.synchronize()
assert int(info.n_records) == n, int(info.n_records)
print("scan_ms", (time.perf_counter() - t0) / reps * 1e3, int(info.n_records), flush=True)
# the C entry point alone (arguments prepared once): what the Python wrapper adds
import ctypes  # noqa: E402
from mgen_amd import _ptr, _stream  # noqa: E402
from mgen_amd._abi import ScanInfo  # noqa: E402
args = (eng.ctx, _ptr(local), local.numel(), SCAN_TCP, _ptr(out[0]), _ptr(out[1]), out[0].numel())
st = _stream(0)
inf = ScanInfo()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(reps):
    eng.lib.mgenx_stream_scan(*args, ctypes.byref(inf), st)
print("c_call_ms", (time.perf_counter() - t0) / reps * 1e3, int(inf.n_records), int(inf.path), flush=True)
# interleaved: wrapper call, C call (median of 40 each)
tw, tc = [], []
for _ in range(40):
    t = time.perf_counter()
    eng.stream_scan(local, SCAN_TCP, out=out)
    tw.append(time.perf_counter() - t)
    t = time.perf_counter()
    eng.lib.mgenx_stream_scan(*args, ctypes.byref(inf), st)
    tc.append(time.perf_counter() - t)
print("interleaved median us: wrapper %.1f C %.1f" % (np.median(tw) * 1e6, np.median(tc) * 1e6),
      flush=True)

# the wrapper's pieces, 2000 calls each (us per call)
def per_call(f, n=2000):
    t = time.perf_counter()
    for _ in range(n):
        f()
    return round((time.perf_counter() - t) / n * 1e6, 2)


print("us: current_stream", per_call(lambda: _stream(0)),
      "raw_stream", per_call(lambda: torch._C._cuda_getCurrentRawStream(0)),
      "slice", per_call(lambda: out[0][:n]),
      "ptr", per_call(lambda: _ptr(local)),
      "info", per_call(ScanInfo),
      "numel", per_call(local.numel), flush=True)
eng.close()
