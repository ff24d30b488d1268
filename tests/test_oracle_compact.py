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


def test_oracle_hint_format(orc):
    """hint_file's layout (the format gck_replay_hints reads; invented here,
    parity unpinned): entries [Timestamp][KeySize][ValueSize][ValuePos][CRC] +
    key, an index entry (hint offset, data offset, check) per HINT_BLOCK entries, a
    32-byte tail; parse_hints walks it and checks index and tail; the CRC
    field is the record header's (kdEntry.CRC, core/keydir.go:3-9)."""
    import struct

    files, names = orc.gen_corpus(seed=61, val_fixed=0, key_min=8, key_max=40, key_universe=300,
                                  tomb_permille=50, max_file_size=1 << 18, n_files=2)
    wf = [files[i] for i in sorted(range(len(files)), key=lambda i: names[i])]
    reset = [True, False]
    recs, _ = orc.replay(wf, reset)
    data, hints = orc.compact(wf, recs, reset, 1 << 15)
    B = orc.HINT_BLOCK
    for d, h in zip(data, hints):
        ents = orc.parse_hints(h)
        n, eb, db, magic, ver = struct.unpack_from("<QQQII", h, len(h) - 32)
        assert (n, db, magic, ver) == (len(ents), len(d), orc.HINT_MAGIC, orc.HINT_VERSION)
        assert len(h) == eb + 24 * ((n + B - 1) // B) + 32
        for ts, key, vs, vpos, crc, rec_off in ents:  # each entry describes its record in the data file
            hcrc, hts, ks, hvs = struct.unpack_from("<IIII", d, rec_off)
            assert (hcrc, hts, ks, hvs) == (crc, ts, len(key), vs)
            assert d[rec_off + 16:rec_off + 16 + ks] == key and vpos == rec_off + 16 + ks
    # an empty merge: one empty data file, a tail-only hint file
    assert orc.hint_file([], 0) == struct.pack("<QQQII", 0, 0, 0, orc.HINT_MAGIC, orc.HINT_VERSION)
    assert orc.parse_hints(orc.hint_file([], 0)) == []
