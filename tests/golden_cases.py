"""Loader + checker for the golden replay fixtures (tests/golden/<case>/).

The checker is shared by the oracle tests (CPU) and the product parity tests
(GPU) so both are held to the same known answers from the reference's tests.
"""
import json
import os
import zlib

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def case_names():
    return sorted(d for d in os.listdir(GOLDEN) if os.path.isdir(os.path.join(GOLDEN, d)))


def load_case(name):
    d = os.path.join(GOLDEN, name)
    meta = json.load(open(os.path.join(d, "case.json")))
    files = [np.fromfile(os.path.join(d, w + ".csk"), dtype=np.uint8) for w in meta["walk"]]
    reset_after = [w != meta["active"] for w in meta["walk"]]
    return meta, files, reset_after


def check_case(meta, files, recs, keydir, status):
    """recs: structured array with REC_DTYPE fields; keydir: {key bytes: rec row};
    status: dict with status, err_off, n_recs, final_last_offset."""
    walk = meta["walk"]
    want_status = 1 if meta["status"] == "unexpected_eof" else 0
    assert status["status"] == want_status, (status, meta["note"])
    der = meta.get("derived", {})
    if "err_off" in der:
        assert status["err_off"] == der["err_off"]
    if "n_recs" in der:
        assert status["n_recs"] == der["n_recs"]
    if "final_last_offset" in meta:
        assert status["final_last_offset"] == meta["final_last_offset"]
    exp = meta["expect"]
    if want_status == 0:
        # the keydir must hold exactly the expected keys (core/keydir.go:59-69 keys())
        assert sorted(keydir.keys()) == sorted(k.encode() for k in exp), meta["note"]
    for k, e in exp.items():
        r = keydir[k.encode()]
        data = files[int(r["file"])]
        if "file" in e:
            assert walk[int(r["file"])] == e["file"], k
        if "value" in e:
            # what Get does: read ValueSize bytes at ValuePos of File (core/db.go:304-313)
            pos, n = int(r["value_pos"]), int(r["value_size"])
            assert bytes(data[pos:pos + n]) == e["value"].encode(), k
            assert int(r["crc"]) == zlib.crc32(e["value"].encode())
        if "crc_ok" in e:
            assert bool(int(r["flags"]) & 2) == e["crc_ok"], k
    for k, e in der.items():
        if k.startswith("_") or not isinstance(e, dict):
            continue
        r = keydir[k.encode()]
        for field, v in e.items():
            assert int(r[field]) == v, (k, field)
    # verdict must agree with an independent zlib CRC of the record's last ValueSize bytes
    for r in recs:
        data = files[int(r["file"])]
        end = int(r["rec_off"]) + 16 + int(r["key_len"]) + (0 if int(r["flags"]) & 1 else int(r["value_size"]))
        v = bytes(data[end - int(r["value_size"]):end])
        assert (zlib.crc32(v) == int(r["crc"])) == bool(int(r["flags"]) & 2)
