"""Boundary phase of the C3 workload: per-chunk chain lengths (records k_walk
follows from each speculative entry) against k_walk's time -- the walk is as
long as its longest chains.   python tools/chunks.py [chunk_kib]"""
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import gocask_amd as g  # noqa: E402

kib = int(sys.argv[1]) if len(sys.argv) > 1 else 0
ctx = g.ReplayContext(chunk_bytes=kib << 10)
ctx.encode(**bench.CONFIGS["c3"])
for _ in range(3):
    ctx.run()
D = g._lib.load_diag()
n = ctx_n = ctypes.c_uint64()
g._lib.check(D.gck_diag_chunks(ctx._h, None, None, 0, ctypes.byref(n)))
cnt = np.zeros(n.value, np.uint32)
ent = np.zeros(n.value, np.uint64)
g._lib.check(D.gck_diag_chunks(ctx._h, cnt.ctypes.data, ent.ctypes.data, n.value, ctypes.byref(n)))
has = ent != np.uint64(0xFFFFFFFFFFFFFFFF)
c = cnt[has]
st = ctx.stats()
print(json.dumps(dict(chunk_kib=kib or 512, chunks=int(n.value), with_entry=int(has.sum()), records=int(c.sum()),
                      mean=round(float(c.mean()), 1), p50=int(np.percentile(c, 50)), p99=int(np.percentile(c, 99)),
                      p999=int(np.percentile(c, 99.9)), max=int(c.max()), boundary_ms=round(st["ms_phase"]["boundary"], 4),
                      fixups=st["n_fixups"])))
ctx.close()
