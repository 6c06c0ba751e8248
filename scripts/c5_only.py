"""Config 5 alone (bench.extra_config5 at world 1) -- for rocprofv3 kernel traces."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from mgen_amd import Engine  # noqa: E402

eng = Engine(0)
print(json.dumps(bench.extra_config5(torch, eng, torch.device("cuda:0"))))
