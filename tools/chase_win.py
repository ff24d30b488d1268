"""Windowed-walk probe (gck_diag_chase_win): 65,536 dependent chains, as many
as k_walk's lanes, each reading a W-byte window per round trip, with the
round trips per chain a C3 walk needs at that window (simulated on the C3
generator: W = 16 B: 156.8 hops per 512 KiB chunk; 128 B: 119.2; 256 B: 83.9;
512 B: 62.3 round trips)."""
import ctypes, json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gocask_amd as g
import bench
ctx = g.ReplayContext()
ctx.encode(**bench.CONFIGS["c3"])
ctx.run()
D = g._lib.load_diag()
D.gck_diag_chase_win.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_uint32, ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
out = {}
ms = ctypes.c_double()
for lpc, hops in ((1, 157), (1, 326), (8, 119), (8, 239), (16, 84), (16, 174), (32, 62), (32, 125)):
    g._lib.check(D.gck_diag_chase_win(ctx._h, lpc, hops, 5, ctypes.byref(ms)))
    out[f"W{16 * lpc}_h{hops}"] = round(ms.value, 4)
print(json.dumps(out))
