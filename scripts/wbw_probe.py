"""Write / read / copy bandwidth of plain torch kernels on an 806 MB buffer (config-3 slab
size): the practical ceilings the pack (writes) and unpack (reads) are compared with."""
import json
import sys

import torch

sys.path.insert(0, ".")
from bench import timed  # noqa: E402

n = 806066437
a = torch.empty(n, dtype=torch.uint8, device="cuda")
b = torch.empty(n, dtype=torch.uint8, device="cuda")
a32 = a[: n // 4 * 4].view(torch.int32)
out = {}
out["fill_u8_ms"] = timed(torch, lambda: a.fill_(0))
out["zero_i32_ms"] = timed(torch, lambda: a32.zero_())
out["copy_ms"] = timed(torch, lambda: b.copy_(a))
out["sum_i32_ms"] = timed(torch, lambda: a32.sum())
for k in list(out):
    out[k] = round(out[k], 4)
out["fill_tbps"] = round(n / out["zero_i32_ms"] / 1e9, 2)
out["copy_tbps_rw"] = round(2 * n / out["copy_ms"] / 1e9, 2)
out["read_tbps"] = round(n / out["sum_i32_ms"] / 1e9, 2)
print(json.dumps(out))
