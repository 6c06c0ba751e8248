"""A plain 1 GiB fill (torch fill_), for the pack's write-path counters to compare with."""
import time

import torch

buf = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")
buf.fill_(1)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(20):
    buf.fill_(1)
torch.cuda.synchronize()
print("fill_ms", (time.perf_counter() - t0) / 20 * 1e3)
