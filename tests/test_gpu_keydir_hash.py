"""Keys hashed in the finalize pass (gck_ctx_keydir_hash): the keydir built
from those hashes must be the oracle's keydir (keyDir.set / unset over every
record in walk order, core/keydir.go:22-49) and the keydir of a run that did
not hash -- Puts whose key sits in the record's header + key registers and
the others (tombstones, keys longer than 28 - (offset mod 4) bytes), with and
without tombstones kept, for a second keydir of the same run, and after the
flag is turned off again."""
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


def _keydirs(g, files, reset, keep):
    with g.ReplayContext() as ctx:
        ctx.load(files, reset)
        ctx.run()
        plain, _ = ctx.keydir(keep_tombstones=keep)
        ctx.keydir_hash(True)
        ctx.run()
        hashed, _ = ctx.keydir(keep_tombstones=keep)
        again, _ = ctx.keydir(keep_tombstones=keep)  # the same run: the kept hashes
        ctx.keydir_hash(False)
        ctx.run()
        off, _ = ctx.keydir(keep_tombstones=keep)
    return plain, hashed, again, off


def _check(g, orc, files, reset, keep):
    plain, hashed, again, off = _keydirs(g, files, reset, keep)
    for other in (hashed, again, off):
        assert np.array_equal(other, plain)
    if not keep:
        want, _ = orc.replay(files, reset)
        kd = orc.keydir(files, want, reset)
        assert len(plain) == len(kd)


@pytest.mark.parametrize("name", case_names())
@pytest.mark.parametrize("keep", [False, True])
def test_keydir_hash_golden(g, orc, name, keep):
    _, files, reset = load_case(name)
    _check(g, orc, files, reset, keep)


@pytest.mark.parametrize("seed,kw", [
    (101, dict(val_fixed=0, key_min=8, key_max=24, key_universe=2000, tomb_permille=100, max_file_size=1 << 20,
               n_files=3)),
    (102, dict(val_fixed=0, key_min=8, key_max=200, key_universe=500, tomb_permille=200, max_file_size=1 << 20,
               n_files=2)),
    (103, dict(val_fixed=17, key_min=9, key_max=31, key_universe=300, tomb_permille=50, flip_permille=50,
               max_file_size=1 << 19, n_files=4)),
])
@pytest.mark.parametrize("keep", [False, True])
def test_keydir_hash_random(g, orc, seed, kw, keep):
    files, names = orc.gen_corpus(seed=seed, **kw)
    walk = sorted(range(len(files)), key=lambda i: names[i])
    wf = [files[i] for i in walk]
    reset = [i + 1 < len(wf) for i in range(len(wf))]
    _check(g, orc, wf, reset, keep)


@pytest.mark.parametrize("hash_first", [False, True])
def test_keydir_table_overflow(g, orc, hash_first):
    """Mostly distinct keys: a fresh context sizes its table for half the
    records, so keys run out of slots (kMaxProbe) and the table is built again
    for every record distinct -- in k_kd_insert, or after the finalize that
    inserted (hash_first); the next runs are sized by the key count.  Every
    keydir equals the oracle's; Get finds every live key and no absent one."""
    files, names = orc.gen_corpus(seed=111, val_fixed=8, key_min=8, key_max=20, key_universe=1 << 40,
                                  tomb_permille=20, max_file_size=1 << 18, n_files=3)
    walk = sorted(range(len(files)), key=lambda i: names[i])
    wf = [files[i] for i in walk]
    reset = [i + 1 < len(wf) for i in range(len(wf))]
    want, _ = orc.replay(wf, reset)
    kd = orc.keydir(wf, want, reset)
    # more keys than the slots of a table sized for half the records (a power
    # of two >= 1.25 n / 2): some must overflow
    slots = 1024
    while slots < len(want) // 2 + len(want) // 8:
        slots *= 2
    assert len(kd) > slots
    with g.ReplayContext() as ctx:
        ctx.load(wf, reset)
        ctx.keydir_hash(hash_first)
        for _ in range(2):  # the first: overflow and rebuild; the second: sized by the count
            ctx.run()
            live, _ = ctx.keydir()
            assert len(live) == len(kd)
            got = {bytes(wf[int(r["file"])][int(r["rec_off"]) + 16:int(r["rec_off"]) + 16 + int(r["key_len"])]):
                   int(r["rec_off"]) for r in live}
            assert got == {k: int(r["rec_off"]) for k, r in kd.items()}
        keys = list(kd)[:500] + [b"absent-key-%d" % i for i in range(100)]
        st, vs, _, _ = ctx.get_batch(keys, values=False)
        assert (st[:500] == 0).all() and (st[500:] == g._lib.GCK_EKEY_NOT_FOUND).all()


@pytest.mark.parametrize("hash_first", [False, True])
def test_keydir_inline_all_ones(g, orc, hash_first):
    """Keys whose 8-byte words are all 0xFF look like a slot word that has not
    landed: those probes compare from the arena.  Keys differing only past
    their first 24 bytes, only in length, or only in a 0xFF word must stay
    distinct; updates and deletes of each keep last-writer-wins (the oracle's
    keydir); Get finds each live key's last value."""
    ff = b"\xff" * 8
    keys = [ff, ff * 2, ff * 3, ff * 3 + b"a", ff * 3 + b"b", ff + b"x" + ff, ff + b"y" + ff, b"k" + ff * 2,
            b"\xff" * 7, b"\xff" * 9, b"p" * 24 + b"tail-1", b"p" * 24 + b"tail-2", b"p" * 24, b"p" * 23]
    recs, ts = [], 1700000000
    for rnd in range(3):
        for i, k in enumerate(keys):
            ts += 1
            if (i + rnd) % 5 == 4:
                recs.append(orc.tombstone(ts, k))
            else:
                recs.append(orc.entry(ts, k, b"v%d-%d" % (rnd, i)))
    files = [np.frombuffer(b"".join(recs), np.uint8)]
    want, _ = orc.replay(files, [False])
    kd = orc.keydir(files, want, [False])
    with g.ReplayContext() as ctx:
        ctx.load(files, [False])
        ctx.keydir_hash(hash_first)
        ctx.run()
        live, _ = ctx.keydir()
        got = {bytes(files[0][int(r["rec_off"]) + 16:int(r["rec_off"]) + 16 + int(r["key_len"])]): int(r["rec_off"])
               for r in live}
        assert got == {k: int(r["rec_off"]) for k, r in kd.items()}
        st, vs, _, vals = ctx.get_batch(keys)
        for k, s, v in zip(keys, st, vals):
            if k in kd:
                assert s == 0
                o = int(kd[k]["value_pos"])
                assert v == bytes(files[0][o:o + int(kd[k]["value_size"])])
            else:
                assert s == g._lib.GCK_EKEY_NOT_FOUND
