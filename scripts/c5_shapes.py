"""Config 5's TCP-rule unpack under the long kernel's shapes (diagnostics build, variant 40-43:
rows per block x threads per workgroup; 0 = the product shape), interleaved; bench.extra_config5
builds, scans and unpacks, and asserts every record decodes without error."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from mgen_amd import Engine  # noqa: E402

eng = Engine(0, diag=True)
out = {}
for rnd in range(2):
    for v in (0, 42, 44, 45):
        eng.set_unpack_variant(v)
        r = bench.extra_config5(torch, eng, torch.device("cuda:0"))
        out.setdefault(str(v), []).append(r["unpack_ms"])
        print(v, r["unpack_ms"], flush=True)
print(json.dumps(out))
