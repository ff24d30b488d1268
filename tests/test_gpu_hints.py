"""Hint-driven replay (gck_replay_hints / gck_ctx_replay_hints, SURVEY.md §8f
f4; the reference's roadmap "merging and hint files", README.md:60): the
tuples of a merged database from its hint files alone must equal, field for
field, the tuples a replay of its data files gives (core/db.go:110-178 with
core/keydir.go:22-34: rec_off, file, KeySize, ValuePos with the carried
lastOffset, ValueSize, CRC, Timestamp), with flags F_HINT (the value is not
read: no CRC verdict) -- for the golden cases' and random corpora's merges,
for several reset patterns (the carried lastOffset), with keys, as the keydir
(live), and for the hints of two merges in one walk; malformed hint files are
refused.  The hint format is invented here (parity unpinned: the reference
has none); the data-file replay it is checked against is pinned."""
import numpy as np
import pytest

from golden_cases import case_names, load_case

pytestmark = pytest.mark.gpu

SAME = ["rec_off", "file", "key_len", "value_pos", "value_size", "crc", "ts"]


@pytest.fixture(scope="module")
def g():
    import __graft_entry__

    __graft_entry__.build()
    import gocask_amd

    assert gocask_amd.device_count() > 0, "no GPU visible"
    return gocask_amd


def _merge(g, files, reset, max_size):
    with g.ReplayContext() as ctx:
        ctx.load(files, reset)
        ctx.run()
        ctx.keydir(fetch=False)
        data, hints, _ = ctx.compact(max_size)
    return [np.asarray(d, np.uint8) for d in data], [np.asarray(h, np.uint8) for h in hints]


def _check(g, data, hints, reset):
    want, wst = g.replay(data, reset, keys=True)
    got, gst = g.replay_hints(hints, reset, keys=True)
    assert gst["status"] == 0 and wst["status"] == 0
    assert len(got) == len(want)
    for f in SAME:
        assert np.array_equal(got[f], want[f]), f
    assert (got["flags"] == g.F_HINT).all() and (got["crc_calc"] == 0).all()
    assert gst["files_walked"] == wst["files_walked"] and gst["final_last_offset"] == wst["final_last_offset"]
    assert np.array_equal(gst["keys"], wst["keys"])
    # the keydir: last entry per key (a merge's hints hold distinct keys)
    lw, _ = g.replay(data, reset, live=True, keys=True)
    lg, lst = g.replay_hints(hints, reset, live=True, keys=True)
    for f in SAME:
        assert np.array_equal(lg[f], lw[f]), f
    return got


def _resets(n):
    yield [True] * n
    yield [i + 1 < n for i in range(n)]  # every file but the active one (core/db.go:117)
    yield [i % 2 == 1 for i in range(n)]  # carried lastOffset across pairs


@pytest.mark.parametrize("name", case_names())
@pytest.mark.parametrize("max_size", [1 << 30, 64])
def test_hints_golden(g, orc, name, max_size):
    _, files, reset = load_case(name)
    recs, st = orc.replay(files, reset)
    if st["status"] != 0:
        pytest.skip("a startup error: no keydir to merge")
    data, hints = _merge(g, files, reset, max_size)
    want_d, want_h = orc.compact(files, recs, reset, max_size)
    assert [bytes(h) for h in hints] == want_h  # the device writes the oracle's hint bytes
    for rs in _resets(len(data)):
        _check(g, data, hints, rs)


@pytest.mark.parametrize("seed,kw,max_size", [
    (81, dict(val_fixed=0, key_min=8, key_max=24, key_universe=3000, tomb_permille=50, max_file_size=4 << 20,
              n_files=4), 1 << 20),
    (82, dict(val_fixed=0, key_min=8, key_max=200, key_universe=500, tomb_permille=100, max_file_size=1 << 20,
              n_files=3), 5000),
    (83, dict(val_fixed=100, key_min=8, key_max=8, key_universe=20000, tomb_permille=0, max_file_size=8 << 20,
              n_files=2), 1 << 30),
])
def test_hints_random(g, orc, seed, kw, max_size):
    files, names = orc.gen_corpus(seed=seed, **kw)
    walk = sorted(range(len(files)), key=lambda i: names[i])
    wf = [files[i] for i in walk]
    reset = [i + 1 < len(wf) for i in range(len(wf))]
    data, hints = _merge(g, wf, reset, max_size)
    for h in hints:  # blocks of GCK_HINT_BLOCK entries, a partial last one
        orc.parse_hints(bytes(h))
    for rs in _resets(len(data)):
        _check(g, data, hints, rs)


def test_hints_two_merges_keydir(g, orc):
    """The hints of two merges in one walk (keys in both): the keydir from the
    hints = the keydir of a replay of both merges' data files."""
    fa, na = orc.gen_corpus(seed=91, val_fixed=0, key_min=8, key_max=16, key_universe=400, tomb_permille=0,
                            max_file_size=1 << 18, n_files=2)
    fb, nb = orc.gen_corpus(seed=92, val_fixed=0, key_min=8, key_max=16, key_universe=400, tomb_permille=0,
                            max_file_size=1 << 18, n_files=2)
    da, ha = _merge(g, fa, [True, True], 1 << 16)
    db, hb = _merge(g, fb, [True, True], 1 << 16)
    data, hints = da + db, ha + hb
    reset = [i + 1 < len(data) for i in range(len(data))]
    lw, _ = g.replay(data, reset, live=True, keys=True)
    lg, _ = g.replay_hints(hints, reset, live=True, keys=True)
    assert len(lg) == len(lw)
    for f in SAME:
        assert np.array_equal(lg[f], lw[f]), f


def test_hints_context(g, orc):
    """gck_ctx_replay_hints on a context: fetch and keydir as after a run;
    Get, scrub and compaction refused (the arena holds no values)."""
    files = _demo(orc)
    data, hints = _merge(g, files, [True, False], 1 << 16)
    want, _ = g.replay(data, [True] * (len(data) - 1) + [False])
    with g.ReplayContext() as ctx:
        ctx.load(hints, [True] * (len(hints) - 1) + [False])
        ms = ctx.replay_hints()
        assert ms >= 0
        got = ctx.fetch()[0]
        for f in SAME:
            assert np.array_equal(got[f], want[f]), f
        live, _ = ctx.keydir()
        assert len(live) == len(want)  # a merge's entries are the live keys
        for bad in (lambda: ctx.scrub_keydir(), lambda: ctx.compact(1 << 20), lambda: ctx.get_batch([b"x"])):
            with pytest.raises(g._lib.GckError):
                bad()


def _demo(orc):
    files, names = orc.gen_corpus(seed=95, val_fixed=0, key_min=8, key_max=24, key_universe=800, tomb_permille=80,
                                  max_file_size=1 << 18, n_files=2)
    order = sorted(range(len(files)), key=lambda i: names[i])
    return [files[i] for i in order]


def test_hints_malformed(g, orc):
    files = _demo(orc)
    _, hints = _merge(g, files, [True, False], 1 << 30)
    h = bytes(hints[0])
    n = int.from_bytes(h[-32:-24], "little")
    B = g._lib.HINT_BLOCK
    assert n > 2 * B + 3  # several blocks, a partial last one
    T, X = 32, 24  # tail, index entry bytes
    ix = len(h) - T - X * ((n + B - 1) // B)  # the index
    first_key = 20  # the first entry's key (after its five header words)
    cases = {
        "truncated": h[:-1],
        "magic": h[:-8] + b"XXXX" + h[-4:],
        "version": h[:-4] + (2).to_bytes(4, "little"),
        "entry count": h[:-T] + (n + 1).to_bytes(8, "little") + h[-T + 8:],
        "key size": h[:4] + (0xFFFF).to_bytes(4, "little") + h[8:],
        "value pos": h[:12] + (int.from_bytes(h[12:16], "little") + 1).to_bytes(4, "little") + h[16:],
        "index": h[:ix + X] + (1).to_bytes(8, "little") + h[ix + X + 8:],
        # well-formed entries whose bytes changed: only the tail's check sees them
        "key byte": h[:first_key] + bytes([h[first_key] ^ 1]) + h[first_key + 1:],
        "timestamp": bytes([h[0] ^ 0x80]) + h[1:],
        "crc": h[:16] + bytes([h[16] ^ 1]) + h[17:],
        "check": h[:ix + X + 16] + bytes([h[ix + X + 16] ^ 1]) + h[ix + X + 17:],
    }
    # a hint file with no entries whose tail claims data-file bytes (they would
    # only feed the carried lastOffset, checked by nothing)
    empty_tail = (0).to_bytes(8, "little") * 2 + (100).to_bytes(8, "little") + h[-8:]
    cases["data bytes without entries"] = empty_tail
    good, _ = g.replay_hints([np.frombuffer(h, np.uint8)], [False])
    assert len(good) == n
    ok_empty, _ = g.replay_hints([np.frombuffer((0).to_bytes(24, "little") + h[-8:], np.uint8)], [False])
    assert len(ok_empty) == 0
    for what, b in cases.items():
        with pytest.raises(g._lib.GckError):
            g.replay_hints([np.frombuffer(b, np.uint8)], [False])


def test_hints_every_single_byte_flip_refused(g, orc):
    # Every byte of a version-3 hint file is covered: entry bytes by their
    # block's integrity word, index entries by the walk (offsets) and the word,
    # the tail by the size checks.  So one flipped bit anywhere must make
    # gck_replay_hints refuse the file -- never return different tuples.
    files = _demo(orc)
    _, hints = _merge(g, files, [True, False], 1 << 30)
    h = bytes(hints[0])
    good, _ = g.replay_hints([np.frombuffer(h, np.uint8)], [False])
    rng = np.random.default_rng(123)
    n_idx = (int.from_bytes(h[-32:-24], "little") + 15) // 16
    ebytes = int.from_bytes(h[-24:-16], "little")
    # positions: every region (entries, index, tail) plus random ones
    pos = [0, 4, 8, 12, 16, 20, ebytes - 1, ebytes, ebytes + 8, ebytes + 16, ebytes + 24 * n_idx - 1,
           len(h) - 32, len(h) - 24, len(h) - 16, len(h) - 8, len(h) - 4, len(h) - 1]
    pos += [int(x) for x in rng.integers(0, len(h), 60)]
    for p in pos:
        bit = 1 << int(rng.integers(0, 8))
        b = bytearray(h)
        b[p] ^= bit
        try:
            got, _ = g.replay_hints([np.frombuffer(bytes(b), np.uint8)], [False])
        except g._lib.GckError:
            continue
        raise AssertionError(f"flip at {p} (bit {bit}) accepted: {len(got)} vs {len(good)} tuples")
