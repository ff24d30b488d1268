"""Random-access probes (gck_diag_stream_pattern 3..14) on the C3 arena: the
walk's hop rate at 8 Ki..256 Ki concurrent chains, dependent vs independent."""
import ctypes, json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gocask_amd as g
import bench
ctx = g.ReplayContext()
ctx.encode(**bench.CONFIGS["c3"])
for _ in range(3):
    ctx.run()
out = {"phase_ms": ctx.stats()["ms_phase"]}
ms, gh = ctypes.c_double(), ctypes.c_double()
for pat in range(3, 15):
    g._lib.check(g._lib.load_diag().gck_diag_stream_pattern(ctx._h, pat, 3, ctypes.byref(ms), ctypes.byref(gh)))
    kind = "dep" if pat < 9 else "indep"
    out[f"{kind}_{8 << ((pat - 3) % 6)}Ki"] = dict(ms=round(ms.value, 3), ghops=round(gh.value, 2))
print(json.dumps(out))
