"""Parity at BASELINE.json's full sizes: the exact C3 and C5 workloads that
bench.py times (16 x 2 GiB rotated files, 32 GiB, Zipf values, 1 % deletes;
C5 adds single-bit flips to 1 % of the values).

The oracle cannot replay 32 GiB in a test's time, so the whole run is checked
through size-independent properties of the corpus spec and of
the reference's replay rules, and walk file 0 (2 GiB, the file bench.py's CPU
baseline replays) is compared field for field with the oracle:

  - the record count equals the encoder's op count, status 0, and
    final_last_offset = the active (last walked) file's length
    (core/db.go:110-123: every other file resets lastOffset);
  - per file the records tile the file exactly: rec_off[0] = 0,
    rec_off[i+1] = rec_off[i] + 16 + key_len + (tombstone ? 0 : ValueSize),
    the last record ends at the file's length (core/db.go:145-178);
  - ValuePos = rec_off + 16 + KeySize mod 2^32 (core/keydir.go:22-34, carry 0);
  - Timestamp = 1700000000 + op, every op exactly once, ops increasing in
    creation order; tombstones exactly the ops the spec deletes (spec.H tag 3);
  - the CRC verdict (core/db.go:311 on every record): no rejects for C3, the
    flipped set for C5; crc_calc == crc exactly for the accepted ones.
"""
import numpy as np
import pytest

import bench
import spec

pytestmark = pytest.mark.gpu

FIELDS = ("rec_off", "file", "key_len", "value_pos", "value_size", "crc", "ts", "flags", "crc_calc")
TS0 = 1700000000


@pytest.fixture(scope="module")
def g():
    import __graft_entry__

    __graft_entry__.build()
    import gocask_amd

    assert gocask_amd.device_count() > 0, "no GPU visible"
    return gocask_amd


def _check_full(g, orc, name):
    kw = dict(bench.CONFIGS[name])
    with g.ReplayContext() as ctx:
        info = ctx.encode(**kw)
        ctx.run()
        got, st = ctx.fetch()
        ctx.run()  # second run: the device-only path, same answers
        got2, st2 = ctx.fetch()
        stats = ctx.stats()
    nf = info["n_files"]
    sizes = [int(info["sizes"][info["walk_order"][w]]) for w in range(nf)]
    assert nf == kw["n_files"] and sum(sizes) > 31 << 30
    assert st["status"] == 0 and len(got) == info["n_ops"]
    assert st["final_last_offset"] == sizes[-1] % (1 << 32)
    assert stats["device_path"] and stats["n_reruns"] == 0
    assert st2 == st
    for f in FIELDS:
        assert np.array_equal(got[f], got2[f]), f

    # records in walk order, files in order, each file tiled exactly
    fidx = got["file"].astype(np.int64)
    assert (np.diff(fidx) >= 0).all() and fidx[0] == 0 and fidx[-1] == nf - 1
    tomb = (got["flags"] & 1) == 1
    off = got["rec_off"].astype(np.uint64)
    klen = got["key_len"].astype(np.uint64)
    vsz = got["value_size"].astype(np.uint64)
    ent = np.uint64(16) + klen + np.where(tomb, np.uint64(0), vsz)
    bounds = np.searchsorted(fidx, np.arange(nf + 1))
    for w in range(nf):
        a, b = bounds[w], bounds[w + 1]
        assert b > a and off[a] == 0
        assert np.array_equal(off[a + 1:b], off[a:b - 1] + ent[a:b - 1]), w
        assert int(off[b - 1] + ent[b - 1]) == sizes[w], w
    ks = np.where(tomb, np.uint64(0), klen)
    assert np.array_equal(got["value_pos"], ((off + np.uint64(16) + ks) % np.uint64(1 << 32)).astype(np.uint32))
    assert np.array_equal(vsz[tomb], klen[tomb])  # Delete: ValueSize = len(key) (core/db.go:245)
    assert ((klen >= kw["key_min"]) & (klen <= kw["key_max"])).all()

    # timestamps: every op once; within a file ops increase by one
    ops = got["ts"].astype(np.int64) - TS0
    assert np.array_equal(np.sort(ops), np.arange(len(got)))
    for w in range(nf):
        a, b = bounds[w], bounds[w + 1]
        assert np.array_equal(np.diff(ops[a:b]), np.ones(b - a - 1, np.int64)), w
    assert np.array_equal(tomb, (spec.H(kw["seed"], 3, ops) % np.uint64(1000)) < np.uint64(kw["tomb_permille"]))

    # the verdict on every record
    ok = (got["flags"] & 2) == 2
    assert np.array_equal(ok, got["crc_calc"] == got["crc"])
    flips = kw.get("flip_permille", 0)
    if flips:
        want_bad = spec.expected_flips(kw["seed"], ops, flips, kw["tomb_permille"])
        assert want_bad.sum() > 50000
        assert np.array_equal(~ok, want_bad)
        assert stats["n_crc_fail"] == int(want_bad.sum())
    else:
        assert ok.all() and stats["n_crc_fail"] == 0

    # walk file 0 (data_0, 2 GiB) against the oracle, field for field
    okw = dict(kw)
    okw["n_files"] = 1
    files, names = orc.gen_corpus(**okw)
    assert len(files[0]) == sizes[0] and names[0].startswith("data_0_")
    want, wst = orc.replay(files, [True])
    assert wst["status"] == 0
    n0 = bounds[1]
    assert len(want) == n0
    for f in FIELDS:
        assert np.array_equal(got[f][:n0], want[f]), f


def test_config3_full_32gib(g, orc):
    _check_full(g, orc, "c3")


def test_config5_full_32gib_reject_set(g, orc):
    _check_full(g, orc, "c5")
