"""C3 keydir scrub (gck_ctx_scrub_keydir) timing, for profiling k_verify."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gocask_amd as g
import bench
ctx = g.ReplayContext()
ctx.encode(**bench.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "c3"])
ctx.run()
ctx.keydir(fetch=False)
for _ in range(3):
    st, cc, bad, ms = ctx.scrub_keydir()
    print("scrub_ms", round(ms, 3), "bad", bad, flush=True)
