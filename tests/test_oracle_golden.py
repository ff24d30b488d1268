"""Pin the CPU oracle before trusting it (CPU-only).

* the reference tests' known answers (tests/golden/, made by make_golden.py);
* the published CRC-32/IEEE check value that Go's hash/crc32 produces;
* the pure-Python restatement as a second opinion on every fixture and on
  small random corpora.
"""
import zlib

import numpy as np
import pytest

from golden_cases import case_names, check_case, load_case


def test_crc_check_values(orc):
    assert orc.crc32(b"123456789") == 0xCBF43926  # CRC-32/ISO-HDLC check value
    assert orc.crc32(b"") == 0
    assert orc.crc32(b"val") == 2548021861  # the CRC core/db_test.go:428-471 stores for "val"
    rng = np.random.default_rng(0)
    for n in [1, 7, 8, 9, 63, 64, 65, 79, 80, 127, 128, 129, 1000, 4097, 65536 + 13]:
        b = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert orc.crc32(b) == zlib.crc32(b)
        assert orc.lib().orc_crc32_fast(np.frombuffer(b, np.uint8).ctypes.data, n) == zlib.crc32(b)
        # the CPU baseline's CLMUL path (Go's amd64 ieeeCLMUL speed class), also at odd addresses
        a = np.frombuffer(b"\0" + b, np.uint8)
        assert orc.lib().orc_crc32_clmul(a.ctypes.data + 1, n) == zlib.crc32(b), n


@pytest.mark.parametrize("name", case_names())
def test_oracle_matches_golden(orc, name):
    meta, files, reset_after = load_case(name)
    recs, status = orc.replay(files, reset_after)
    kd = orc.keydir(files, recs, reset_after)
    check_case(meta, files, recs, kd, status)


@pytest.mark.parametrize("name", case_names())
def test_python_restatement_agrees(orc, name):
    meta, files, reset_after = load_case(name)
    recs, status = orc.replay(files, reset_after)
    precs, pkd, pstatus, plast = orc.replay_py(files, reset_after)
    assert status["status"] == pstatus["status"]
    assert len(precs) == len(recs)
    for a, b in zip(recs, precs):
        assert int(a["rec_off"]) == b["rec_off"] and int(a["value_pos"]) == b["value_pos"]
        assert int(a["crc_calc"]) == b["crc_calc"] and bool(int(a["flags"]) & 2) == b["crc_ok"]
    assert status["final_last_offset"] == plast


def test_random_corpora_agree(orc):
    for seed, kw in [(3, dict(val_fixed=0, key_min=8, key_max=24, key_universe=300, tomb_permille=50,
                              flip_permille=100, max_file_size=1 << 18, n_files=3)),
                     (4, dict(val_fixed=100, key_min=8, key_max=8, n_ops=500, max_file_size=1 << 14))]:
        files, names = orc.gen_corpus(seed=seed, **kw)
        walk = sorted(range(len(files)), key=lambda i: names[i])
        wf = [files[i] for i in walk]
        active = max(names)
        reset = [names[i] != active for i in walk]
        recs, status = orc.replay(wf, reset)
        precs, pkd, pstatus, plast = orc.replay_py(wf, reset)
        assert len(recs) == len(precs) > 0
        assert [int(r["crc_calc"]) for r in recs] == [p["crc_calc"] for p in precs]
        kd = orc.keydir(wf, recs, reset)
        assert sorted(kd) == sorted(pkd)
        assert all(int(kd[k]["rec_off"]) == pkd[k]["rec_off"] for k in kd)
        # flips are confined to values, so rejects == flipped records exactly
        assert status["status"] == 0


def test_baseline_counts(orc):
    files, names = orc.gen_corpus(seed=5, val_fixed=0, key_min=8, key_max=24, key_universe=200,
                                  tomb_permille=20, max_file_size=1 << 18, n_files=2)
    recs, status = orc.replay(files, [True, True])
    kd = orc.keydir(files, recs, [True, True])
    live, bst = orc.baseline(files, [True, True])
    assert live == len(kd) and bst["n_recs"] == status["n_recs"]
    assert bst["final_last_offset"] == status["final_last_offset"]


def test_lexical_walk_order():
    # internal/fs/disk.go:122-145 + filepath.Walk sorts names bytewise
    names = [f"data_{n}_{1700000000 + n}.csk" for n in range(16)]
    order = [int(n.split("_")[1]) for n in sorted(names)]
    assert order == [0, 10, 11, 12, 13, 14, 15, 1, 2, 3, 4, 5, 6, 7, 8, 9]
