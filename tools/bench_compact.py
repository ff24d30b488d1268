"""Compaction (gck_ctx_compact) timing on a BASELINE config: replay, keydir,
then merge the live records into new files + hint files (row f4)."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gocask_amd as g
import bench
cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
ctx = g.ReplayContext()
ctx.encode(**bench.CONFIGS[cfg])
ctx.run()
n_live, _ = ctx.keydir(fetch=False)
runs = [ctx.compact(2 << 30, fetch=False) for _ in range(4)]
nf, nd, nh, _ = runs[-1]
ms = [r[3] for r in runs[1:]]
best = min(ms)
# algorithmic traffic: every live record read once and written once, hint entries written
print(json.dumps({"cfg": cfg, "live_records": n_live, "merged_files": nf, "data_bytes": nd, "hint_bytes": nh,
                  "ms": [round(x, 3) for x in ms], "GBps_algorithmic": round((2 * nd + nh) / best / 1e6, 1)}))
