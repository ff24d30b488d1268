"""Merge (compaction) and hint files on the device (the
reference's roadmap item "merging and hint files", README.md:60), through the
C-ABI, against the oracle's restatement (oracle.compact): the live records in
walk order, Put into a fresh database with MaxDataFileSize (core/db.go:185-231),
record bytes verbatim, plus Bitcask hint entries.  Round trip: replaying the
merged files gives the same live keys and values, and the hint entries equal
the replay's (Timestamp, key, ValueSize, ValuePos)."""
import numpy as np
import pytest

from golden_cases import case_names, load_case

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def g():
    import __graft_entry__

    __graft_entry__.build()
    import gocask_amd

    assert gocask_amd.device_count() > 0, "no GPU visible"
    return gocask_amd


def _compact(g, files, reset, max_size):
    with g.ReplayContext() as ctx:
        ctx.load(files, reset)
        ctx.run()
        ctx.keydir(fetch=False)
        data, hints, _ = ctx.compact(max_size)
    return [bytes(d) for d in data], [bytes(h) for h in hints]


def _roundtrip(g, orc, data, hints, want_kd, files):
    """Replay of the merged files: same live keys and values; hints = replay."""
    got_recs, st = g.replay([np.frombuffer(d, np.uint8) for d in data] or [np.zeros(0, np.uint8)],
                            [True] * max(len(data), 1))
    assert st["status"] == 0
    assert not (got_recs["flags"] & 1).any()  # no tombstones survive a merge
    by_key = {}
    for r in got_recs:
        d = data[int(r["file"])]
        o = int(r["rec_off"])
        key = d[o + 16:o + 16 + int(r["key_len"])]
        assert key not in by_key  # one record per live key
        by_key[key] = (r, d[int(r["value_pos"]):int(r["value_pos"]) + int(r["value_size"])])
    assert set(by_key) == set(want_kd)
    for key, w in want_kd.items():  # the record's own value (ValuePos may carry the active-file quirk)
        o = int(w["rec_off"]) + 16 + int(w["key_len"])
        assert by_key[key][1] == bytes(files[int(w["file"])][o:o + int(w["value_size"])])
    for k, h in enumerate(hints):
        ents = orc.parse_hints(h)
        recs_k = [r for r in got_recs if int(r["file"]) == k]
        assert [(e[0], e[1], e[2], e[3]) for e in ents] == [
            (int(r["ts"]), by_key_key(data[k], r), int(r["value_size"]), int(r["value_pos"])) for r in recs_k]


def by_key_key(d, r):
    o = int(r["rec_off"])
    return d[o + 16:o + 16 + int(r["key_len"])]


@pytest.mark.parametrize("name", case_names())
@pytest.mark.parametrize("max_size", [1 << 30, 64, 17])
def test_compact_golden(g, orc, name, max_size):
    _, files, reset = load_case(name)
    recs, st = orc.replay(files, reset)
    if st["status"] != 0:
        pytest.skip("a startup error: no keydir to merge")
    want_d, want_h = orc.compact(files, recs, reset, max_size)
    got_d, got_h = _compact(g, files, reset, max_size)
    assert got_d == want_d
    assert got_h == want_h
    _roundtrip(g, orc, got_d, got_h, orc.keydir(files, recs, reset), files)


@pytest.mark.parametrize("seed,kw,max_size", [
    (71, dict(val_fixed=0, key_min=8, key_max=24, key_universe=2000, tomb_permille=50, max_file_size=4 << 20,
              n_files=4), 1 << 20),
    (72, dict(val_fixed=100, key_min=8, key_max=8, key_universe=50, tomb_permille=200, max_file_size=1 << 18,
              n_files=6), 1000),
    (73, dict(val_fixed=0, key_min=8, key_max=200, key_universe=300, tomb_permille=100, flip_permille=100,
              max_file_size=1 << 20, n_files=3), 1 << 16),
    (74, dict(val_fixed=0, key_min=8, key_max=24, key_universe=100000, tomb_permille=10,
              max_file_size=64 << 20, n_files=2), 1 << 30),
])
def test_compact_random(g, orc, seed, kw, max_size):
    files, names = orc.gen_corpus(seed=seed, **kw)
    walk = sorted(range(len(files)), key=lambda i: names[i])
    wf = [files[i] for i in walk]
    reset = [i + 1 < len(wf) for i in range(len(wf))]
    recs, _ = orc.replay(wf, reset)
    want_d, want_h = orc.compact(wf, recs, reset, max_size)
    got_d, got_h = _compact(g, wf, reset, max_size)
    assert len(got_d) == len(want_d)
    for a, b in zip(got_d, want_d):
        assert a == b
    assert got_h == want_h
    _roundtrip(g, orc, got_d, got_h, orc.keydir(wf, recs, reset), wf)


def test_compact_first_record_over_limit(g, orc):
    # a first live record larger than MaxDataFileSize: the fresh database's
    # first file is rotated away empty (core/db.go:214-231)
    big = orc.entry(1, b"k1", b"v" * 100) + orc.entry(2, b"k2", b"w" * 10)
    files = [np.frombuffer(big, np.uint8)]
    recs, _ = orc.replay(files, [False])
    want_d, want_h = orc.compact(files, recs, [False], 50)
    assert want_d[0] == b""
    got_d, got_h = _compact(g, files, [False], 50)
    assert got_d == want_d and got_h == want_h


def test_compact_requires_puts_only(g, orc):
    _, files, reset = load_case(case_names()[0])
    with g.ReplayContext() as ctx:
        ctx.load(files, reset)
        ctx.run()
        ctx.keydir(keep_tombstones=True, fetch=False)
        with pytest.raises(Exception):
            ctx.compact(1 << 20)


@pytest.mark.parametrize("seed,vmin,max_size", [
    (81, 0, 64),     # thousands of merged files: the pointer-doubling rotation points
    (82, 0, 17),     # a file per record
    (83, 40, 30),    # every record over the limit: an empty first file, then one file per record
])
def test_compact_many_files(g, orc, seed, vmin, max_size):
    rng = np.random.default_rng(seed)
    ops = []
    for i in range(3000):
        k = b"k%d" % int(rng.integers(0, 900))
        if rng.random() < 0.05:
            ops.append(orc.tombstone(1_700_000_000 + i, k))
        else:
            ops.append(orc.entry(1_700_000_000 + i, k, rng.bytes(int(rng.integers(vmin, vmin + 30)))))
    files = [np.frombuffer(b"".join(ops), np.uint8)]
    recs, st = orc.replay(files, [False])
    assert st["status"] == 0
    want_d, want_h = orc.compact(files, recs, [False], max_size)
    assert len(want_d) > 256  # past the one-wavefront search
    got_d, got_h = _compact(g, files, [False], max_size)
    assert len(got_d) == len(want_d)
    assert got_d == want_d
    assert got_h == want_h


def test_compact_refuses_stale_keydir(g, orc):
    # a run invalidates the keydir: compacting without a fresh gck_ctx_keydir
    # would merge nothing and report success
    _, files, reset = load_case(case_names()[0])
    with g.ReplayContext() as ctx:
        ctx.load(files, reset)
        ctx.run()
        ctx.keydir(fetch=False)
        ctx.compact(1 << 20)  # fresh keydir: fine
        ctx.run()
        with pytest.raises(g._lib.GckError) as e:
            ctx.compact(1 << 20)
        assert e.value.code == g._lib.GCK_EINVAL


def test_compact_refuses_startup_error(g, orc):
    # the reference refuses to open a database whose replay hit a startup
    # error (core/db.go:134-138): there is no keydir to merge
    good = orc.entry(1, b"user", b"alice")
    bad = good + orc.entry(2, b"key", b"value")[:17]  # header + 1 of 3 key bytes: ErrUnexpectedEOF
    files = [np.frombuffer(bad, np.uint8)]
    _, st = orc.replay(files, [False])
    assert st["status"] == 1
    with g.ReplayContext() as ctx:
        ctx.load(files, [False])
        assert ctx.run() == 1
        ctx.keydir(fetch=False)
        with pytest.raises(g._lib.GckError) as e:
            ctx.compact(1 << 20)
        assert e.value.code == g._lib.GCK_EINVAL
