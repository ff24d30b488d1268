"""Device keydir build (gck_ctx_keydir) on C3: device ms of three builds."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import gocask_amd as g  # noqa: E402

ctx = g.ReplayContext()
ctx.encode(**bench.CONFIGS["c3"])
ctx.run()
for _ in range(3):
    ctx.run()  # the first keydir of a run hashes every key
    n, ms = ctx.keydir(fetch=False)
    _, again = ctx.keydir(fetch=False)  # the same run: hashes kept
    print("keydir_ms", round(ms, 3), "rebuild_ms", round(again, 3), "live", n, flush=True)
