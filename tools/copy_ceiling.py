"""Device copy ceiling for the encoder's traffic shape: 1 GiB read + 1 GiB
written by torch's copy kernel, HIP events, best of 10."""
import json

import torch

a = torch.randint(0, 256, (1 << 30,), dtype=torch.uint8, device="cuda")
b = torch.empty_like(a)
for _ in range(3):
    b.copy_(a)
torch.cuda.synchronize()
best = 1e9
for _ in range(10):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    b.copy_(a)
    e1.record()
    e1.synchronize()
    best = min(best, e0.elapsed_time(e1))
print(json.dumps({"copy_ms": round(best, 4), "GBps_read_plus_write": round(2 * (1 << 30) / best / 1e6, 1)}))
