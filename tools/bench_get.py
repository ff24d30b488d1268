"""Batched DB.Get with values (gck_ctx_get_batch, row f3) on the C3 corpus:
65,536 random live keys (their bytes read back from the device arena), the
device time of lookup + CRC + value copy (the API's events), best of 5.
Prints one JSON line."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import gocask_amd as g  # noqa: E402

nkeys = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
ctx = g.ReplayContext()
ctx.encode(**bench.CONFIGS["c3"])
ctx.run()
recs, _ = ctx.keydir()
rng = np.random.default_rng(7)
pick = recs[rng.choice(len(recs), nkeys, replace=False)]
keys = [ctx.read_file(int(r["file"]), int(r["rec_off"]) + 16, int(r["key_len"])).tobytes() for r in pick]
best, vbytes = 1e9, 0
for _ in range(5):
    st, vs, cc, vals = ctx.get_batch(keys, values=True)
    assert (st == 0).all(), np.unique(st)
    best = min(best, ctx.last_get_ms)
    vbytes = int(vs.sum())
for r, v in zip(pick[:64], vals[:64]):  # the values are the replay's records
    assert len(v) == int(r["value_size"])
print(json.dumps({"keys": nkeys, "value_bytes": vbytes, "get_ms": round(best, 4),
                  "GBps_values": round(vbytes / best / 1e6, 1)}))
