"""Config 3 alone (bench.extra_config3) -- pack + unpack timing, for A/B and traces."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from mgen_amd import Engine  # noqa: E402

eng = Engine(0)
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 1):
    print(json.dumps(bench.extra_config3(torch, eng, torch.device("cuda:0"))), flush=True)
