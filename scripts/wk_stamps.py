"""Resident worker, receive path (mgenx_worker_recv: Unpack + the receive checksum): the call's
host-side time next to the wave's own stamps (diagnostics build: header parsed, checksum done,
reply stored, in 10-ns ticks from the poll that saw the request), per message size; also
Unpack alone and ComputeCRC32 alone.  Prints one JSON object."""
import ctypes
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mgen_amd import Engine  # noqa: E402
from mgen_amd.workloads import udp_fixed  # noqa: E402
from oracle import oracle as O  # noqa: E402

eng = Engine(0, diag=True)
w = eng.worker()
out = {"device_mailbox": w.device_mailbox()}
st = (ctypes.c_uint32 * 8)()
for size in (64, 256, 1024, 1472, 4096, 8192):
    tmpl, pool, desc = udp_fixed(2, size)
    slab, _ = O.udp_pack_batch(tmpl, desc, pool, 2 * size, stride=size, checksum=True)
    msg = slab[:size].tobytes()
    for _ in range(200):
        w.recv(msg)
    host, dev = [], []
    for _ in range(2000):
        t = time.perf_counter()
        _, c = w.recv(msg)
        host.append(time.perf_counter() - t)
        eng.lib.mgenx_diag_worker_stamps(w.w, st)
        dev.append((st[0], st[1], st[2], st[4], st[5]))
        assert c is not None
    dd = np.median(np.array(dev, dtype=np.float64), axis=0)
    d = dd * 0.01
    tu = []
    for _ in range(2000):
        t = time.perf_counter()
        w.unpack(msg)
        tu.append(time.perf_counter() - t)
    tc = []
    for _ in range(2000):
        t = time.perf_counter()
        w.crc32(msg[:-4], 0)
        tc.append(time.perf_counter() - t)
    out[str(size)] = {"recv_us": round(np.median(host) * 1e6, 2),
                      "wave_parsed_us": round(d[0], 2), "wave_crc_done_us": round(d[1], 2),
                      "wave_reply_us": round(d[2], 2),
                      "wave_clocks_to_parse": int(dd[3]), "wave_clocks_to_reply": int(dd[4]),
                      "sclk_mhz": round(dd[4] / max(d[2], 1e-3), 0),
                      "unpack_us": round(np.median(tu) * 1e6, 2),
                      "crc32_us": round(np.median(tc) * 1e6, 2)}
w.close()
eng.close()
print(json.dumps(out))
