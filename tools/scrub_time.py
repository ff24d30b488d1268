"""Per-group cycle stamps of a k_verify timing variant (crc_calc carries them:
lane 0 = metadata loads, 1 = the lane path (values <= 256 B), 2 = the wave
path (larger values), 3 = cycles since the previous group ended, 4 = large
values in the group)."""
import json, os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gocask_amd as g
import bench
ctx = g.ReplayContext()
ctx.encode(**bench.CONFIGS["c3"])
ctx.run()
ctx.keydir(fetch=False)
ctx.scrub_keydir()
st, cc, bad, ms = ctx.scrub_keydir()
cc = np.asarray(cc, dtype=np.uint32)
n = len(cc) // 64 * 64
out = dict(ms=round(ms, 3), groups=n // 64)
q = lambda a: [round(float(np.percentile(a, p)), 0) for p in (10, 50, 90, 99)]
for k, name in enumerate(("meta", "lane_path", "wave_path", "between", "n_large")):
    a = cc[k:n:64].astype(np.float64)
    out[name + "_p10_50_90_99"] = q(a)
    out[name + "_sum_per_wave_us"] = round(float(a.sum()) / 4096 / 2000.0, 1) if name != "n_large" else None
print(json.dumps(out))
