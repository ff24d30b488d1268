"""Chain-walk variants on the C3 corpus (gck_diag_walk_variant): stage
stores as built (mode 0), an 8-byte stage (2), no stage stores (4)."""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import gocask_amd as g  # noqa: E402

chunk = int(sys.argv[1]) << 10 if len(sys.argv) > 1 else 0
ctx = g.ReplayContext(chunk_bytes=chunk)
ctx.encode(**bench.CONFIGS["c3"])
ctx.run()
ctx.run()
st = ctx.stats()
out = dict(chunk_kib=chunk >> 10, phases={k: round(v, 3) for k, v in st["ms_phase"].items()})
L = g._lib.load()
ms = ctypes.c_double()
for mode in (0, 2, 4, 0, 2, 4):
    g._lib.check(L.gck_diag_walk_variant(ctx._h, mode, 5, ctypes.byref(ms)))
    out.setdefault(f"walk_mode{mode}", []).append(round(ms.value, 4))
print(json.dumps(out))
