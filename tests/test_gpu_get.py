"""Batched DB.Get and keydir scrub on the device, through the
C-ABI, against DB.Get's semantics (core/db.go:287-316) applied to the oracle's
keydir: empty key -> ErrInvalidKey, absent / deleted -> ErrKeyNotFound, a read
past the file's end -> a file-system error, CRC of the ValueSize bytes at
ValuePos of File != the entry's CRC -> ErrCRCFailed, else the value.  The
golden fixtures add the reference tests' own known answers (values, CRC
failures)."""
import zlib

import numpy as np
import pytest

from golden_cases import case_names, load_case

pytestmark = pytest.mark.gpu

OK, EIO, NOT_FOUND, CRC_FAILED, INVALID_KEY = 0, 5, 6, 7, 8


@pytest.fixture(scope="module")
def g():
    import __graft_entry__

    __graft_entry__.build()
    import gocask_amd

    assert gocask_amd.device_count() > 0, "no GPU visible"
    return gocask_amd


def _keydir(files, recs):
    kd, deleted = {}, set()
    for r in recs:
        o = int(r["rec_off"]) + 16
        key = bytes(files[int(r["file"])][o:o + int(r["key_len"])])
        if int(r["flags"]) & 1:
            kd.pop(key, None)
            deleted.add(key)
        else:
            kd[key] = r
            deleted.discard(key)
    return kd, deleted


def _expected(files, kd, key):
    """(status, value or None, crc or None) of DB.Get(key)."""
    if len(key) == 0:
        return INVALID_KEY, None, None
    r = kd.get(key)
    if r is None:
        return NOT_FOUND, None, None
    f = files[int(r["file"])]
    pos, n = int(r["value_pos"]), int(r["value_size"])
    if pos + n > len(f):
        return EIO, None, None
    val = bytes(f[pos:pos + n])
    crc = zlib.crc32(val)
    return (OK, val, crc) if crc == int(r["crc"]) else (CRC_FAILED, None, crc)


def _queries(kd, deleted, rng, extra=50):
    live = list(kd)
    q = live + sorted(deleted) + [b""]
    for i in range(extra):  # absent keys, including prefixes / extensions of live ones
        if live and i % 2:
            k = live[int(rng.integers(len(live)))]
            q.append(k[:-1] if i % 4 == 1 else k + b"x")
        else:
            q.append(b"absent-%d" % i)
    rng.shuffle(q)
    return q


def _check(files, kd, q, st, vs, cc, vals):
    for i, key in enumerate(q):
        est, ev, ecrc = _expected(files, kd, key)
        assert st[i] == est, (key, st[i], est)
        if est in (OK, CRC_FAILED):
            assert cc[i] == ecrc, key
            assert vs[i] == int(kd[key]["value_size"])
        if vals is not None:
            assert vals[i] == ev, key


def _run(g, files, reset, rng, recs, keep_tombstones=False, values=True):
    """recs: the oracle's records of the corpus (the expectation's keydir)."""
    with g.ReplayContext() as ctx:
        ctx.load(files, reset)
        ctx.run()
        ctx.keydir(keep_tombstones=keep_tombstones, fetch=False)
        kd, deleted = _keydir(files, recs)
        q = _queries(kd, deleted, rng)
        st, vs, cc, vals = ctx.get_batch(q, values=values)
        sst, scc, bad, _ = ctx.scrub_keydir()
        live, _ = ctx.keydir(keep_tombstones=keep_tombstones)
    _check(files, kd, q, st, vs, cc, vals)
    return kd, live, sst, scc, bad


@pytest.mark.parametrize("name", case_names())
def test_get_batch_golden(g, orc, name):
    meta, files, reset = load_case(name)
    rng = np.random.default_rng(1)
    want, _ = orc.replay(files, reset)
    _run(g, files, reset, rng, want)
    # the reference tests' known answers: values Get returns, CRC failures
    with g.ReplayContext() as ctx:
        ctx.load(files, reset)
        ctx.run()
        ctx.keydir(fetch=False)
        keys = [k.encode() for k in meta["expect"]]
        st, _, _, vals = ctx.get_batch(keys)
    for i, (k, e) in enumerate(meta["expect"].items()):
        if "value" in e:
            assert st[i] == OK and vals[i] == e["value"].encode(), k
        if e.get("crc_ok") is False:
            assert st[i] == CRC_FAILED, k


@pytest.mark.parametrize("seed,kw", [
    (61, dict(val_fixed=0, key_min=8, key_max=24, key_universe=2000, tomb_permille=50, flip_permille=50,
              max_file_size=4 << 20, n_files=4)),
    (62, dict(val_fixed=100, key_min=8, key_max=8, key_universe=50, tomb_permille=200, max_file_size=1 << 18,
              n_files=6)),
    (63, dict(val_fixed=0, key_min=8, key_max=200, key_universe=300, tomb_permille=100, flip_permille=100,
              max_file_size=1 << 20, n_files=3)),
])
def test_get_batch_and_scrub_random(g, orc, seed, kw):
    files, names = orc.gen_corpus(seed=seed, **kw)
    walk = sorted(range(len(files)), key=lambda i: names[i])
    wf = [files[i] for i in walk]
    reset = [i + 1 < len(wf) for i in range(len(wf))]
    rng = np.random.default_rng(seed)
    want, _ = orc.replay(wf, reset)
    for keep in (False, True):  # the table is the same either way; only the live list differs
        kd, live, sst, scc, bad = _run(g, wf, reset, rng, want, keep_tombstones=keep, values=not keep)
        # scrub: Get of every entry gck_ctx_keydir returned, in its order
        for i, r in enumerate(live):
            o = int(r["rec_off"]) + 16
            key = bytes(wf[int(r["file"])][o:o + int(r["key_len"])])
            if int(r["flags"]) & 1:
                continue  # a kept tombstone: its "value" is read like any entry's
            est, _, ecrc = _expected(wf, kd, key)
            assert sst[i] == est, (i, key)
            if est != EIO:
                assert scc[i] == ecrc
        if not keep:
            assert bad == sum(1 for k in kd if _expected(wf, kd, k)[0] != OK)
            if kw.get("flip_permille"):
                assert bad > 0  # flipped values are caught


def test_get_batch_c3_shape_scrub_counts(g):
    # C3 shape at 1/64 scale with 1 % bit flips: the scrub's rejects are
    # exactly the live entries whose replay verdict (GCK_F_CRC_OK) is a reject
    kw = dict(seed=3, val_fixed=0, key_min=8, key_max=24, key_universe=80000, tomb_permille=10,
              flip_permille=10, max_file_size=32 << 20, n_files=16)
    with g.ReplayContext() as ctx:
        ctx.encode(**kw)
        ctx.run()
        live, _ = ctx.keydir()
        st, cc, bad, ms = ctx.scrub_keydir()
    # every value of a live entry lies inside its record (no carry quirk in
    # this corpus), so Get's CRC equals the replay's
    assert np.array_equal(cc, live["crc_calc"])
    assert bad == int(np.count_nonzero((live["flags"] & 2) == 0)) and bad > 0
    assert np.array_equal(st == CRC_FAILED, (live["flags"] & 2) == 0)


def test_get_batch_requires_keydir(g, orc):
    files, _ = orc.gen_corpus(seed=64, val_fixed=10, key_min=8, key_max=8, key_universe=10,
                              max_file_size=1 << 12, n_files=1)
    with g.ReplayContext() as ctx:
        ctx.load(files, [False])
        ctx.run()
        with pytest.raises(Exception):
            ctx.get_batch([b"k"])
        ctx.keydir(fetch=False)
        ctx.get_batch([b"k"])
        ctx.run()  # a new run invalidates the keydir
        with pytest.raises(Exception):
            ctx.get_batch([b"k"])


@pytest.mark.parametrize("vlen", [1, 3, 4, 5, 16, 1020, 1021, 1022, 1023, 1024, 1025, 1028, 2047, 2048, 2049, 65536])
def test_get_batch_value_lengths(g, orc, vlen):
    # the device CRC splits a value into 1 KiB stripes (padding in front) and
    # folds the 0xFFFFFFFF init into its first 4 bytes: every edge of that
    files, _ = orc.gen_corpus(seed=65, val_fixed=vlen, key_min=8, key_max=12, key_universe=40, flip_permille=100,
                              max_file_size=max(1 << 16, 48 * (vlen + 28)), n_files=1)
    want, _ = orc.replay(files, [False])
    _run(g, files, [False], np.random.default_rng(vlen), want)


def _mix64d(x):
    """kd_common.h mix64d on a numpy uint64 array (wrapping arithmetic)."""
    x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


def _key_hash8(ids):
    """kd_common.h key_hash of the 8-byte keys struct.pack('<Q', id)."""
    with np.errstate(over="ignore"):
        h = np.full(ids.shape, np.uint64(0x9E3779B97F4A7C15) ^ np.uint64(8 << 32), dtype=np.uint64)
        h = _mix64d(h ^ (ids & np.uint64(0xFFFFFFFF)))
        h = _mix64d(h ^ (ids >> np.uint64(32))) + np.uint64(1)
        return _mix64d(h)


@pytest.mark.parametrize("hashed", [False, True])
def test_keydir_clustered_hashes(g, orc, hashed):
    # 400 keys whose hashes share their low 12 bits: every table the build
    # sizes (1024..4096 slots) puts them on one home slot, so the bounded
    # builds (256 probes) overflow and the last build probes without a bound,
    # as the reference's Go map takes any key set (core/keydir.go:22-34).
    # The keydir and Get must still be exact, the lookups probing as far as
    # the build did.
    import struct

    cand = np.arange(1, 3_000_000, dtype=np.uint64)
    ids = cand[(_key_hash8(cand) & np.uint64(0xFFF)) == 0][:400]
    assert len(ids) == 400
    keys = [struct.pack("<Q", int(i)) for i in ids]
    rng = np.random.default_rng(7)
    blob, t = bytearray(), 1700000000
    for k in keys:  # every key once, then a third of them again (the later record wins)
        blob += orc.entry(t, k, rng.bytes(int(rng.integers(1, 40))))
        t += 1
    for k in keys[::3]:
        blob += orc.entry(t, k, rng.bytes(int(rng.integers(1, 40))))
        t += 1
    for k in keys[1::7]:
        blob += orc.tombstone(t, k)
        t += 1
    files, reset = [np.frombuffer(bytes(blob), dtype=np.uint8)], [False]
    want, _ = orc.replay(files, reset)
    kd, deleted = _keydir(files, want)
    with g.ReplayContext() as ctx:
        ctx.load(files, reset)
        if hashed:
            ctx.keydir_hash(True)
        ctx.run()
        live, _ = ctx.keydir()
        assert ctx.stats()["kd_longest_probe"] > 256
        q = _queries(kd, deleted, rng)
        st, vs, cc, vals = ctx.get_batch(q)
    assert len(live) == len(kd)
    got = {bytes(files[0][int(r["rec_off"]) + 16:int(r["rec_off"]) + 16 + int(r["key_len"])]): int(r["rec_off"])
           for r in live}
    assert got == {k: int(r["rec_off"]) for k, r in kd.items()}
    _check(files, kd, q, st, vs, cc, vals)
