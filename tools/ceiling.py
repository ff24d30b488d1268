#!/usr/bin/env python3
"""k_crc_rows against the stream-read ceilings on the resident C3 arena, one box.

  python tools/ceiling.py [--reps 3] [--secs 2.0]
  (with GCK_LIB_PATH=gocask_amd/var/libgocask_hip_clk.so, the stamps build of
   tools/clock.py, also k_crc_rows' own per-XCD end times and clocks)

Interleaved per repetition: the replay step (k_crc_rows by its HIP events),
the static grid-stride stream read bench.py reports since round 2
(gck_diag_stream_read), and the XCD-balanced stream read with k_crc_rows' work
assignment (gck_diag_stream_blocks: 64-row blocks; 4/8 of the rounds static as
k_crc_rows, also all-queue and all-static).  Then one stamped pass of the
balanced read after >= --secs of back-to-back passes: per-XCD median end time
and shader clock (by the wavefronts' XCC ids).  One JSON line.
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


def stamp_stats(st, xcc):
    s = st.astype(np.float64)
    ok = (s[:, 1] > 0) & (s[:, 3] > s[:, 1])
    s, x = s[ok], xcc[ok]
    t0 = s[:, 1].min()
    end = (s[:, 3] - t0) / 100.0  # us (real time at 100 MHz)
    ghz = (s[:, 2] - s[:, 0]) / (s[:, 3] - s[:, 1]) * 0.1
    xs = sorted(set(int(v) for v in x))
    return dict(waves=int(len(s)), clock_ghz_median=round(float(np.median(ghz)), 3),
                end_us_p50=round(float(np.median(end)), 1), end_us_max=round(float(end.max()), 1),
                xcd_end_us_p50={k: round(float(np.median(end[x == k])), 1) for k in xs},
                xcd_end_us_max={k: round(float(end[x == k].max()), 1) for k in xs},
                xcd_ghz={k: round(float(np.median(ghz[x == k])), 3) for k in xs})


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--secs", type=float, default=2.0)
    ap.add_argument("--config", default="c3")
    args = ap.parse_args()
    import torch  # noqa: F401  (the runtime first, as bench.py)
    import bench
    import gocask_amd as g
    from gocask_amd import _lib

    ctx = g.ReplayContext(device=0)
    ctx.encode(**bench.CONFIGS[args.config])
    nbytes = ctx.stats()["bytes"] if ctx.stats().get("bytes") else None
    for _ in range(3):
        ctx.run()
    rows = []
    for rep in range(args.reps):
        s0 = ctx.stats()
        t0 = time.perf_counter()
        for _ in range(10):
            ctx.run()
        torch.cuda.synchronize()
        step = (time.perf_counter() - t0) / 10 * 1e3
        s1 = ctx.stats()
        nbytes = s1["bytes"]
        r = dict(rep=rep, step_ms=round(step, 3), crc_rows_ms=round((s1["ms_crc_rows_sum"] - s0["ms_crc_rows_sum"]) / 10, 4))
        r["stream_read_ms"] = round(ctx.stream_read_ceiling(10)[0], 4)
        for e in (4, 0, 8):
            r[f"blocks{e}_ms"] = round(ctx.stream_blocks_ceiling(10, e)[0], 4)
        rows.append(r)
    out = {"config": args.config, "bytes": nbytes, "lib": os.path.basename(_lib.LIB_PATH), "reps": rows}
    med = {k: float(np.median([r[k] for r in rows])) for k in rows[0] if k != "rep"}
    out["median_ms"] = {k: round(v, 4) for k, v in med.items()}
    out["crc_rows_over_balanced"] = round(med["crc_rows_ms"] / med["blocks4_ms"], 4)
    out["balanced_gbs"] = round(nbytes / (med["blocks4_ms"] * 1e-3) / 1e9, 1)
    # stamped balanced read after back-to-back passes (steady clock)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < args.secs:
        ctx.stream_blocks_ceiling(20, 4)
    ms, _ = ctx.stream_blocks_ceiling(5, 4, stamp=True)
    st, xcc = ctx.clock_stamps()
    out["blocks4_stamped"] = dict(stamp_stats(st, xcc), pass_ms=round(ms, 4))
    # k_crc_rows' own stamps when this is the stamps build
    L = _lib.load()
    if hasattr(L, "gck_xp_clock_xcc"):
        L.gck_xp_clock_read.argtypes = [ctypes.c_int, ctypes.c_void_p]
        L.gck_xp_clock_xcc.argtypes = [ctypes.c_int, ctypes.c_void_p]
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < args.secs:
            ctx.run()
        L.gck_xp_clock_reset()
        ctx.run()
        buf = np.zeros(4 * L.gck_xp_clock_waves(), dtype=np.uint64)
        xb = np.zeros(L.gck_xp_clock_waves(), dtype=np.uint32)
        assert L.gck_xp_clock_read(0, buf.ctypes.data) == 0
        assert L.gck_xp_clock_xcc(0, xb.ctypes.data) == 0
        out["crc_rows_stamped"] = stamp_stats(buf.reshape(-1, 4), xb)
    print(json.dumps(out), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
