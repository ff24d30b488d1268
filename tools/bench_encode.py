"""Throughput of gck_encode_batch (row f4) on a device-resident batch.

  python tools/bench_encode.py [--gib 2] [--iters 5]

Synthetic records: 8-24 B keys, bounded Zipf-like values (64 B .. 64 KiB,
mostly small; most bytes in large values), 1 % deletes, all generated on the
device.  Prints one JSON line: payload bytes in + record bytes out per second
(algorithmic traffic = key + value bytes read + record bytes written)."""
import argparse
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np
import torch

from gocask_amd import _lib


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=2.0)
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    rng = np.random.default_rng(1)
    target = int(a.gib * 2**30)
    # value sizes: 64 * 2^(Zipf-ish exponent), capped at 64 KiB
    est = target // 3000 + 16
    vlen = np.minimum(64 << rng.geometric(0.35, est).clip(1, 10) - 1, 65536).astype(np.uint64)
    vlen = vlen[: int(np.searchsorted(np.cumsum(vlen), target)) + 1]
    n = len(vlen)
    klen = rng.integers(8, 25, n).astype(np.uint64)
    tomb = (rng.random(n) < 0.01).astype(np.uint8)
    koff = np.zeros(n + 1, np.uint64)
    voff = np.zeros(n + 1, np.uint64)
    koff[1:] = np.cumsum(klen)
    voff[1:] = np.cumsum(vlen)
    dev = torch.device("cuda", 0)
    keys = torch.randint(0, 256, (int(koff[-1]),), dtype=torch.uint8, device=dev)
    vals = torch.randint(0, 256, (int(voff[-1]),), dtype=torch.uint8, device=dev)
    d_koff = torch.from_numpy(koff.view(np.int64)).to(dev)
    d_voff = torch.from_numpy(voff.view(np.int64)).to(dev)
    d_ts = torch.arange(n, dtype=torch.int32, device=dev)
    d_tomb = torch.from_numpy(tomb).to(dev)
    payload = int(koff[-1]) + int((vlen * (1 - tomb)).sum())
    out_bytes = 16 * n + payload
    out = torch.empty(out_bytes, dtype=torch.uint8, device=dev)
    out_off = torch.empty(n + 1, dtype=torch.int64, device=dev)
    total = ctypes.c_uint64(0)
    L = _lib.load()
    stream = torch.cuda.current_stream(dev).cuda_stream

    def run():
        _lib.check(L.gck_encode_batch(keys.data_ptr(), d_koff.data_ptr(), vals.data_ptr(), d_voff.data_ptr(),
                                      d_ts.data_ptr(), d_tomb.data_ptr(), n, out.data_ptr(), out_bytes,
                                      out_off.data_ptr(), ctypes.byref(total), stream))

    run()
    torch.cuda.synchronize()
    ts = []
    for _ in range(a.iters):
        t0 = time.perf_counter()
        run()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    best = min(ts)
    traffic = payload + out_bytes
    print(json.dumps({"records": n, "payload_bytes": payload, "out_bytes": int(total.value),
                      "ms_best": round(best * 1e3, 3), "ms_all": [round(t * 1e3, 3) for t in ts],
                      "GBps_algorithmic": round(traffic / best / 1e9, 1),
                      "note": "wall time per call: device offsets (scan), one 16 B readback, the encode kernel"}))


if __name__ == "__main__":
    main()
