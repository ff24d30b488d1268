"""Which chunks does speculation get wrong on the C3 corpus, and why
(gck_diag_spec_entries): prints each mismatch with the headers at both
positions."""
import ctypes
import os
import struct
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import gocask_amd as g  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
chunk = int(sys.argv[2]) << 10 if len(sys.argv) > 2 else 0
ctx = g.ReplayContext(chunk_bytes=chunk)
info = ctx.encode(**bench.CONFIGS[cfg])
ctx.run()
L = g._lib.load()
n = ctypes.c_uint64()
L.gck_diag_spec_entries(ctx._h, None, None, 0, ctypes.byref(n))
spec = np.zeros(n.value, np.uint64)
fin = np.zeros(n.value, np.uint64)
g._lib.check(L.gck_diag_spec_entries(ctx._h, spec.ctypes.data, fin.ctypes.data, n.value, ctypes.byref(n)))
bad = np.nonzero(spec != fin)[0]
cb = chunk or (512 << 10)
sizes = [int(info["sizes"][info["walk_order"][w]]) for w in range(info["n_files"])]
first = np.cumsum([0] + [(s + cb - 1) // cb for s in sizes])
print(f"{len(bad)} of {n.value} chunks mis-speculated")
NONE = (1 << 64) - 1
for c in bad[:20]:
    f = int(np.searchsorted(first, c, side="right") - 1)
    cs = (int(c) - int(first[f])) * cb
    def hdr(p):
        if p == NONE:
            return None
        b = ctx.read_file(f, p, 16)
        return struct.unpack("<IIII", bytes(b))
    s, t = int(spec[c]), int(fin[c])
    print(f"chunk {c} file {f} start {cs}: spec {s if s != NONE else None} (+{s - cs if s != NONE else ''}) "
          f"hdr {hdr(s)} | final {t if t != NONE else None} (+{t - cs if t != NONE else ''}) hdr {hdr(t)}")

# follow chain_ok (kHops + 1 headers) from each wrong entry, as k_spec_entry does
for c in bad[:5]:
    f = int(np.searchsorted(first, c, side="right") - 1)
    q = int(spec[c])
    ln = sizes[f]
    hops = []
    for h in range(5):
        if q == ln or q + 16 > ln:
            hops.append(("end", q))
            break
        crc, ts, ks, vs = struct.unpack("<IIII", bytes(ctx.read_file(f, q, 16)))
        klen = ks if ks else vs
        nxt = q + 16 + ks + vs
        hops.append((q, ks, vs, klen, nxt, nxt <= ln))
        q = nxt
    print("chain", c, hops)
