"""CPU check of the oracle's merge restatement (oracle.compact): replaying the
merged files with the oracle gives the same live keys and values as the
original keydir, every merged file respects MaxDataFileSize unless it holds a
single oversized record, and the hint entries equal the replay's
(Timestamp, key, ValueSize, ValuePos)."""
import numpy as np
import pytest

from golden_cases import case_names, load_case


@pytest.mark.parametrize("name", case_names())
@pytest.mark.parametrize("max_size", [1 << 30, 64, 17])
def test_oracle_compact_roundtrip(orc, name, max_size):
    _, files, reset = load_case(name)
    recs, st = orc.replay(files, reset)
    if st["status"] != 0:
        pytest.skip("a startup error: no keydir to merge")
    # the record's own value bytes (a merge copies records verbatim; the
    # keydir's ValuePos may carry the active-file quirk, core/db.go:117-119)
    def val(r):
        o = int(r["rec_off"]) + 16 + int(r["key_len"])
        return bytes(files[int(r["file"])][o:o + int(r["value_size"])])
    want = {k: val(r) for k, r in orc.keydir(files, recs, reset).items()}
    data, hints = orc.compact(files, recs, reset, max_size)
    assert len(data) == len(hints) >= 1
    for d in data:
        assert len(d) <= max_size or orc.replay([np.frombuffer(d, np.uint8)], [True])[1]["n_recs"] == 1
    arrs = [np.frombuffer(d, np.uint8) for d in data]
    got_recs, gst = orc.replay(arrs, [True] * len(arrs))
    assert gst["status"] == 0 and gst["n_recs"] == len(want)
    got = {}
    for r in got_recs:
        d = data[int(r["file"])]
        o = int(r["rec_off"])
        got[d[o + 16:o + 16 + int(r["key_len"])]] = d[int(r["value_pos"]):int(r["value_pos"]) + int(r["value_size"])]
    assert got == want
    ents = [e for h in hints for e in orc.parse_hints(h)]
    assert [(e[0], e[2], e[3]) for e in ents] == [(int(r["ts"]), int(r["value_size"]), int(r["value_pos"]))
                                                  for r in got_recs]
