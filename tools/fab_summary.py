"""Summarise tools/xp_fused_ab.sh runs: k_fuse full / listed and k_crc_rows
launch durations (ms) per tag and repetition, from the rocprofv3 databases."""
import collections
import glob
import sqlite3
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
for d in sorted(glob.glob(f"{root}/fab_*_*/")):
    dbs = glob.glob(d + "**/*.db", recursive=True)
    if not dbs:
        continue
    db = sqlite3.connect(dbs[0])
    cols = [r[1] for r in db.execute("pragma table_info(kernels)")]
    rows = sorted((dict(zip(cols, r)) for r in db.execute("select * from kernels")), key=lambda r: r["start"])
    t = collections.defaultdict(list)
    for r in rows:
        n = r["name"]
        ms = round((r["end"] - r["start"]) / 1e6, 3)
        if "k_fuse<" in n:
            t["fuse_full" if r["grid_x"] > 16384 else "fuse_listed"].append(ms)
        elif "k_crc_rows<0" in n:
            t["crc_rows"].append(ms)
        elif "k_finalize" in n:
            t["finalize"].append(ms)
    print(d.split("/")[-2], {k: v for k, v in t.items()})
