"""Debug: whole-stream scans of test_config5's stream on fresh / reused engines."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from mgen_amd import SCAN_TCP, Engine, to_device  # noqa: E402
from streams import golden, tcp_stream  # noqa: E402

gold = golden()
rng = np.random.default_rng(0x4D47454E + 5)
s = tcp_stream(gold, np.full(4096, 16384), rng)
d = to_device(s)
from streams import sink_stream  # noqa: E402
from mgen_amd import SCAN_SINK  # noqa: E402
for label, pre in [("fresh", None), ("after-small", 300), ("after-big", 20000), ("ovf-sink", -1),
                   ("ovf-tcp", -2)]:
    eng = Engine(0)
    if pre and pre > 0:
        s2 = tcp_stream(gold, rng.integers(76, 5000, pre), rng)
        eng.stream_scan(to_device(s2), SCAN_TCP)
    elif pre:
        r2 = np.random.default_rng(0x4D47454E + 70 + (1 if pre == -1 else 0))
        if pre == -1:
            a = sink_stream(gold, r2.integers(28, 8193, 250), r2)
            b = sink_stream(gold, r2.integers(28, 8193, 250), r2)
        else:
            a = tcp_stream(gold, r2.integers(76, 5000, 400), r2)
            b = tcp_stream(gold, r2.integers(76, 5000, 400), r2)
        s2 = np.concatenate([a, np.full(70_000, 2, np.uint8), b])
        for _ in range(2):
            o2, l2, i2 = eng.stream_scan(to_device(s2), SCAN_SINK if pre == -1 else SCAN_TCP)
            print("pre", int(i2.n_records), int(i2.resolved), int(i2.candidates), flush=True)
    for k in range(3):
        offs, lens, info = eng.stream_scan(d, SCAN_TCP)
        print(label, k, int(info.n_records), int(info.consumed), int(info.resolved),
              int(info.candidates), flush=True)
    eng.close()
