#!/usr/bin/env python3
"""In-kernel clocks and wavefront timing of every phase of one replay step
(the stamps build: GCK_LIB_PATH=gocask_amd/var/libgocask_hip_clk.so, built by
make -C gocask_amd/csrc OUT=../var/libgocask_hip_clk.so BUILD=build_clk
EXTRA=-DGCK_CLOCK_STAMPS ../var/libgocask_hip_clk.so).

  python tools/phase_clock.py [--secs 2.0]   -> one JSON line

After >= --secs of back-to-back C3 replays, one more replay with stamps: per
kernel (every wavefront of k_spec_entry, k_walk, k_compact, k_crc_rows,
k_finalize, up to 65,536) the median shader clock, the span from the first
wavefront's start to the last one's end, and the wavefront durations.
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

KINDS = {0: "k_crc_rows", 2: "k_spec_entry", 3: "k_walk", 4: "k_compact", 5: "k_finalize"}


def summary(st):
    s = st.astype(np.float64)
    ok = (s[:, 1] > 0) & (s[:, 3] > s[:, 1])
    s = s[ok]
    if not len(s):
        return dict(waves=0)
    t0 = s[:, 1].min()
    dur = (s[:, 3] - s[:, 1]) / 100.0
    ghz = (s[:, 2] - s[:, 0]) / (s[:, 3] - s[:, 1]) * 0.1
    end = (s[:, 3] - t0) / 100.0
    return dict(waves=int(len(s)), clock_ghz_median=round(float(np.median(ghz)), 3),
                span_us=round(float(end.max()), 1), start_us_max=round(float(((s[:, 1] - t0) / 100.0).max()), 1),
                wave_us_p50=round(float(np.median(dur)), 1), wave_us_p90=round(float(np.percentile(dur, 90)), 1),
                wave_us_max=round(float(dur.max()), 1), wave_us_p10=round(float(np.percentile(dur, 10)), 1),
                end_us_p50=round(float(np.median(end)), 1),
                start_us_p50=round(float(np.median((s[:, 1] - t0) / 100.0)), 1),
                start_us_p90=round(float(np.percentile((s[:, 1] - t0) / 100.0, 90)), 1),
                t0_realtime=int(t0))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--secs", type=float, default=2.0)
    ap.add_argument("--config", default="c3")
    args = ap.parse_args()
    import torch  # noqa: F401
    import bench
    import gocask_amd as g
    from gocask_amd import _lib

    L = _lib.load()
    if not hasattr(L, "gck_xp_clock_xcc"):
        raise SystemExit(f"{_lib.LIB_PATH} is not the stamps build")
    L.gck_xp_clock_read.argtypes = [ctypes.c_int, ctypes.c_void_p]
    ctx = g.ReplayContext(device=0)
    ctx.encode(**bench.CONFIGS[args.config])
    ctx.run()
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < args.secs:
        ctx.run()
    L.gck_xp_clock_reset()
    ctx.run()
    out = {"config": args.config, "step_ms": round(ctx.stats()["ms_total"], 3)}
    starts = {}
    for k, name in KINDS.items():
        buf = np.zeros(4 * L.gck_xp_clock_waves(), dtype=np.uint64)
        assert L.gck_xp_clock_read(k, buf.ctypes.data) == 0
        out[name] = summary(buf.reshape(-1, 4))
        starts[name] = out[name].pop("t0_realtime", None)
    if hasattr(L, "gck_xp_fin_split"):
        L.gck_xp_fin_split.argtypes = [ctypes.c_void_p]
        fs = np.zeros(2 * L.gck_xp_clock_waves(), dtype=np.uint64)
        assert L.gck_xp_fin_split(fs.ctypes.data) == 0
        fs = fs.reshape(-1, 2).astype(np.float64)
        fs = fs[fs.sum(axis=1) > 0]
        if len(fs):
            out["k_finalize"]["split_cycles_median"] = dict(wait=float(np.median(fs[:, 0])),
                                                            compute=float(np.median(fs[:, 1])))
    base = min(v for v in starts.values() if v)
    for name, v in starts.items():
        if v:
            out[name]["start_us_in_step"] = round((v - base) / 100.0, 1)
    print(json.dumps(out), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
