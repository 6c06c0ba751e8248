"""pcap2mgen stage timing (bench.extra_pcap's workload): the whole device pipeline, then its
stages one by one (flow-table create / destroy, parse, unpack, lookup, reduce, text)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mgen_amd import Engine  # noqa: E402
from mgen_amd.pcap import Pcap2Mgen  # noqa: E402
from mgen_amd.workloads import pcap_capture  # noqa: E402

n = 1 << 20
eng = Engine(0)
buf, pkt_off, _ = pcap_capture(eng, n)
p = Pcap2Mgen(eng, analytics=True, window=0.25)
p.run_device(buf, pkt_off, n, 1, 0)
torch.cuda.synchronize()


def t(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


print("whole", round(t(lambda: p.run_device(buf, pkt_off, n, 1, 0)), 3), flush=True)


def table():
    tb = eng.flow_table(n)
    eng.flow_table_destroy(tb)


print("table create+destroy (max_flows = n)", round(t(table), 3), flush=True)
pr = eng.pcap_parse(buf, pkt_off, n, 1, 0)
print("parse", round(t(lambda: eng.pcap_parse(buf, pkt_off, n, 1, 0)), 3), flush=True)
print("unpack", round(t(lambda: eng.unpack(buf, n, rec_off=pr["udp_off"], rec_len=pr["udp_len"],
                                           opts=4, ext=True)), 3), flush=True)
q = Pcap2Mgen(eng, analytics=False, window=0.25)
print("no analytics", round(t(lambda: q.run_device(buf, pkt_off, n, 1, 0)), 3), flush=True)
