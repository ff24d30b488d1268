"""Device keydir build (gck_ctx_keydir) on C3: device ms of three builds."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import gocask_amd as g  # noqa: E402

ctx = g.ReplayContext()
ctx.encode(**bench.CONFIGS["c3"])
ctx.run()
ctx.phase_timing(True)
for hashed in (False, True, False, True):
    ctx.keydir_hash(hashed)  # on: the run's finalize hashes the keys
    for _ in range(2):
        ctx.run()
        st = ctx.stats()
        n, ms = ctx.keydir(fetch=False)
        _, again = ctx.keydir(fetch=False)  # the same run: hashes kept
        print("finalize_hash", int(hashed), "finalize_ms", round(st["ms_phase"]["finalize"], 4),
              "keydir_ms", round(ms, 3), "rebuild_ms", round(again, 3), "live", n, flush=True)
