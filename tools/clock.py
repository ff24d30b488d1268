#!/usr/bin/env python3
"""In-kernel clock of k_crc_rows and of a plain non-temporal stream read on the
same resident C3 arena (MI355X_MICROARCH.md DVFS item 6).

Needs the diagnostic build with stamps:
  make -C gocask_amd/csrc OUT=../var/libgocask_hip_clk.so BUILD=build_clk \
       EXTRA=-DGCK_CLOCK_STAMPS ../var/libgocask_hip_clk.so
  GCK_LIB_PATH=gocask_amd/var/libgocask_hip_clk.so python tools/clock.py [--secs 2.5]

Per kernel: >= --secs of back-to-back launches, then the stamps of one more
launch: per wavefront (shader clock, 100 MHz real time) at its loop start and
end; clock = d(clock) / d(real time) x 100 MHz, median over wavefronts.  One
JSON line.
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def stats(L, which, waves_per_wg):
    buf = np.zeros(4 * L.gck_xp_clock_waves(), dtype=np.uint64)
    assert L.gck_xp_clock_read(which, buf.ctypes.data_as(ctypes.c_void_p)) == 0
    s = buf.reshape(-1, 4).astype(np.float64)
    ok = (s[:, 1] > 0) & (s[:, 3] > s[:, 1])
    wg = np.nonzero(ok)[0] // waves_per_wg
    s = s[ok]
    # wave end times from the first wave's start (us); per XCD (workgroups go
    # round-robin over the 8 XCDs) the median end and the median clock
    t0 = s[:, 1].min()
    end = (s[:, 3] - t0) / 100.0
    beg = (s[:, 1] - t0) / 100.0
    xcd = wg % 8
    ghz_all = (s[:, 2] - s[:, 0]) / (s[:, 3] - s[:, 1]) * 0.1
    extra = dict(end_us_p10=round(float(np.percentile(end, 10)), 1), end_us_p50=round(float(np.median(end)), 1),
                 end_us_p90=round(float(np.percentile(end, 90)), 1), end_us_p99=round(float(np.percentile(end, 99)), 1),
                 start_us_p99=round(float(np.percentile(beg, 99)), 1),
                 xcd_end_us_p50=[round(float(np.median(end[xcd == x])), 1) for x in range(8)],
                 xcd_ghz=[round(float(np.median(ghz_all[xcd == x])), 3) for x in range(8)])
    dt, dr = s[:, 2] - s[:, 0], s[:, 3] - s[:, 1]
    ghz = dt / dr * 0.1  # real time ticks at 100 MHz
    wave_us = dr / 100.0
    return dict(waves=int(len(s)), clock_ghz_median=round(float(np.median(ghz)), 4),
                clock_ghz_p10=round(float(np.percentile(ghz, 10)), 4),
                clock_ghz_p90=round(float(np.percentile(ghz, 90)), 4),
                wave_us_median=round(float(np.median(wave_us)), 1), wave_us_max=round(float(wave_us.max()), 1),
                span_us=round(float((s[:, 3].max() - s[:, 1].min()) / 100.0), 1), **extra)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--secs", type=float, default=2.5)
    ap.add_argument("--config", default="c3")
    args = ap.parse_args()
    import torch  # noqa: F401  (the runtime first, as bench.py)
    import bench
    import gocask_amd as g
    from gocask_amd import _lib

    L = _lib.load()
    for n in ("gck_xp_clock_reset", "gck_xp_clock_read", "gck_xp_clock_stream"):
        if not hasattr(L, n):
            raise SystemExit(f"{_lib.LIB_PATH} is not the stamps build (no {n})")
    L.gck_xp_clock_read.argtypes = [ctypes.c_int, ctypes.c_void_p]
    L.gck_xp_clock_stream.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
    ctx = g.ReplayContext(device=0)
    ctx.encode(**bench.CONFIGS[args.config])
    out = {"lib": os.path.basename(_lib.LIB_PATH), "config": args.config}
    # k_crc_rows: back-to-back replays, then the stamps of one more
    ctx.run()
    t0 = time.perf_counter()
    n = 0
    while time.perf_counter() - t0 < args.secs:
        ctx.run()
        n += 1
    s0 = ctx.stats()
    L.gck_xp_clock_reset()
    ctx.run()
    st = ctx.stats()
    out["crc_rows"] = dict(stats(L, 0, 16), warm_runs=n, kernel_ms=round(st["ms_crc_rows_sum"] - s0["ms_crc_rows_sum"], 4),
                           step_ms=round(st["ms_total"], 3))
    # the stream read: back-to-back, then one stamped batch
    ms = ctypes.c_double()
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < args.secs:
        L.gck_xp_clock_stream(ctx._h, 50, ctypes.byref(ms))
    L.gck_xp_clock_reset()
    L.gck_xp_clock_stream(ctx._h, 1, ctypes.byref(ms))
    one = ms.value
    L.gck_xp_clock_stream(ctx._h, 20, ctypes.byref(ms))
    out["stream_read"] = dict(stats(L, 1, 4), kernel_ms=round(ms.value, 4), kernel_ms_stamped_launch=round(one, 4),
                              gbs=round(st["bytes"] / (ms.value * 1e-3) / 1e9, 1))
    print(json.dumps(out), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
