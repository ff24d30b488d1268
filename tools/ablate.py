"""Ablation timing of k_crc_rows variants (diagnostic; not part of the bench)."""
import ctypes, json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gocask_amd as g
cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
import bench
ctx = g.ReplayContext()
ctx.encode(**bench.CONFIGS[cfg])
for _ in range(3):
    ctx.run()
st = ctx.stats()
out = {"cfg": cfg, "bytes": st["bytes"], "phase_ms": st["ms_phase"], "stream": ctx.stream_read_ceiling(5)}
ms = ctypes.c_double()
for mode in [int(x) for x in (sys.argv[2].split(",") if len(sys.argv) > 2 else "0,2,4,6,8,12".split(","))]:
    g._lib.check(ctx._L.gck_diag_crc_variant(ctx._h, mode, 5, ctypes.byref(ms)))
    out[f"mode{mode}_ms"] = round(ms.value, 3)
    out[f"mode{mode}_gbs"] = round(st["bytes"] / ms.value / 1e6, 1)
gbs = ctypes.c_double()
for pat in [0, 1, 2, 15, 16, 17]:
    g._lib.check(ctx._L.gck_diag_stream_pattern(ctx._h, pat, 5, ctypes.byref(ms), ctypes.byref(gbs)))
    out[f"stream_pattern{pat}_ms"] = round(ms.value, 3)
print(json.dumps(out))
