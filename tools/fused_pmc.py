"""One standard and one fused C3 replay (for PMC comparisons of k_crc_rows vs k_fuse)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gocask_amd as g
import bench
for flags in (0, g.core.OPT_FUSED):
    ctx = g.ReplayContext(flags=flags)
    ctx.encode(**bench.CONFIGS["c3"])
    ctx.run()
    ctx.run()
    print(flags, ctx.stats()["ms_phase"], flush=True)
    ctx.close()
