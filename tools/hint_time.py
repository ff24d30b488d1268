"""Hint-driven replay against the full replay on C3's merge (row f4).

C3 is replayed, its keydir merged into 2 GiB data files + hint files
(gck_ctx_compact); then, device-resident: gck_ctx_replay_hints over the hint
files against gck_ctx_run over the merged data files (device ms, 3 runs each);
host-in/host-out: gck_replay_hints against gck_replay (wall ms)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import gocask_amd as g  # noqa: E402


def main():
    ctx = g.ReplayContext()
    ctx.encode(**bench.CONFIGS["c3"])
    ctx.run()
    ctx.keydir(fetch=False)
    data, hints, cms = ctx.compact(2 << 30)
    ctx.close()
    reset = [i + 1 < len(data) for i in range(len(data))]
    out = dict(merged_files=len(data), data_bytes=int(sum(d.size for d in data)),
               hint_bytes=int(sum(h.size for h in hints)), compact_ms=round(cms, 3))
    with g.ReplayContext() as h:
        h.load(hints, reset)
        hm = [h.replay_hints() for _ in range(3)]
        n_h = h.stats()["n_recs"]
    with g.ReplayContext() as d:
        d.load(data, reset)
        d.phase_timing(True)
        dm = []
        for _ in range(4):  # (the first run sizes the record table: not counted)
            d.run()
            dm.append(d.stats()["ms_phase"]["pipeline"])
        dm = dm[1:]
    out.update(hints_device_ms=[round(x, 3) for x in hm], replay_device_ms=[round(x, 3) for x in dm], n_hint_recs=n_h)
    t = time.perf_counter()
    hr, _ = g.replay_hints(hints, reset)
    out["hints_host_ms"] = round((time.perf_counter() - t) * 1e3, 1)
    t = time.perf_counter()
    dr, _ = g.replay(data, reset)
    out["replay_host_ms"] = round((time.perf_counter() - t) * 1e3, 1)
    out["records"] = len(dr)
    out["same"] = bool(len(hr) == len(dr) and all((hr[f] == dr[f]).all() for f in
                                                  ["rec_off", "file", "key_len", "value_pos", "value_size", "crc", "ts"]))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
