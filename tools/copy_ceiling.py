"""Read+write ceiling for the copy-shaped secondary kernels (encoder,
compaction): device-to-device copies of 1 GiB and 8 GiB on one MI355X (torch
copy_, i.e. the runtime's copy kernel), ms and GB/s counting the bytes read
plus the bytes written.  One JSON line per size."""
import json

import torch


def main():
    for gib in (1, 8):
        n = gib << 30
        a = torch.empty(n, dtype=torch.uint8, device="cuda")
        b = torch.empty(n, dtype=torch.uint8, device="cuda")
        a.fill_(1)
        for _ in range(3):
            b.copy_(a)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 10
        e0.record()
        for _ in range(reps):
            b.copy_(a)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        print(json.dumps(dict(gib=gib, ms=round(ms, 4), rw_gbs=round(2 * n / (ms * 1e-3) / 1e9, 1))), flush=True)
        del a, b


if __name__ == "__main__":
    main()
