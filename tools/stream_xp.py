#!/usr/bin/env python3
"""Bytes in flight vs stream rate on the C3 arena (round 6): gck_diag_stream_xp
over rows in flight per wavefront (pf), occupancy (workgroup size, LDS per
workgroup, workgroups per CU) and assignment (64-row blocks or strided rows),
beside the two ceilings bench.py reports.  One JSON line per configuration.

  python tools/stream_xp.py [--iters 5]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--modes", action="store_true", help="only the block assignments (static, queue, split) with stamps")
    args = ap.parse_args()
    import torch  # noqa: F401
    import bench
    import gocask_amd as g
    from gocask_amd import _lib

    from ceiling import stamp_stats
    ctx = g.ReplayContext(device=0)
    ctx.encode(**bench.CONFIGS["c3"])
    ctx.run()
    import torch
    n_cu = torch.cuda.get_device_properties(0).multi_processor_count
    if args.modes:
        for rep in range(3):
            cfgs = [(1, 1, 1024, 160, 1), (1, 2, 1024, 160, 1), (1, 3, 1024, 160, 1),
                    (2, 1, 1024, 160, 1), (2, 2, 1024, 160, 1), (2, 3, 1024, 160, 1),
                    (1, 2, 256, 0, 8), (1, 3, 256, 0, 8)]
            if os.environ.get("XP_SCATTER"):  # static with a round's blocks scattered over the CUs
                cfgs = [(1, 1, 1024, 160, 1), (1, 2, 1024, 160, 1), (1, 3, 1024, 160, 1), (1, 6, 1024, 160, 1),
                        (1, 7, 1024, 160, 1), (3, 1, 256, 160, 1), (3, 6, 256, 160, 1), (3, 7, 256, 160, 1)]
            if os.environ.get("XP_FEW"):  # fewer wavefronts per CU, more rows in flight each
                cfgs = [(1, 1, 1024, 160, 1), (1, 2, 1024, 160, 1),
                        (3, 1, 512, 160, 1), (3, 2, 512, 160, 1), (3, 3, 512, 160, 1),
                        (3, 1, 256, 160, 1), (3, 2, 256, 160, 1), (2, 2, 512, 160, 1)]
            for cfg in cfgs:
                pf, blocks, threads, lds, wpc = cfg
                t, gb = ctx.stream_xp(pf, blocks, threads, lds, wpc, args.iters, stamp=True)
                st, xcc = ctx.clock_stamps()
                w = threads // 64 * wpc * n_cu
                print(json.dumps(dict(rep=rep, kind="xp", pf=pf, blocks=blocks, threads=threads, lds_kib=lds,
                                      wg_per_cu=wpc, ms=round(t, 4), gbs=round(gb, 1),
                                      stamps=stamp_stats(st[:w], xcc[:w]))), flush=True)
        ctx.close()
        return
    for rep in range(2):
        print(json.dumps(dict(rep=rep, kind="stream_read", ms=round(ctx.stream_read_ceiling(args.iters)[0], 4))), flush=True)
        print(json.dumps(dict(rep=rep, kind="stream_blocks", ms=round(ctx.stream_blocks_ceiling(args.iters)[0], 4))), flush=True)
        # (pf, blocks, threads, lds_kib, wg_per_cu): waves per CU = threads/64 x resident workgroups
        for cfg in [(1, 1, 1024, 160, 1), (2, 1, 1024, 160, 1), (3, 1, 1024, 160, 1),
                    (1, 0, 1024, 160, 1), (2, 0, 1024, 160, 1),
                    (1, 1, 1024, 80, 2), (2, 1, 1024, 80, 2),
                    (1, 1, 256, 0, 8), (2, 1, 256, 0, 8), (1, 0, 256, 0, 8), (2, 0, 256, 0, 8)]:
            pf, blocks, threads, lds, wpc = cfg
            t, gb = ctx.stream_xp(pf, blocks, threads, lds, wpc, args.iters, stamp=True)
            line = dict(rep=rep, kind="xp", pf=pf, blocks=blocks, threads=threads, lds_kib=lds, wg_per_cu=wpc,
                        ms=round(t, 4), gbs=round(gb, 1))
            w = threads // 64 * wpc * n_cu
            if w <= 16384:  # (the stamps hold 16,384 wavefronts)
                st, xcc = ctx.clock_stamps()
                line["stamps"] = stamp_stats(st[:w], xcc[:w])
            print(json.dumps(line), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
