"""Parity of the HIP replay path against the CPU oracle (GPU box only).

Everything goes through the C-ABI (libgocask_hip.so).  Bit-exact bar: every
field of every record tuple, the CRC accept/reject verdict, the keydir, the
error status and keyDir.lastOffset must equal the oracle's.
"""
import os
import struct
import zlib

import numpy as np
import pytest

import oracle as orc_mod
from golden_cases import case_names, check_case, load_case

pytestmark = pytest.mark.gpu

FIELDS = ("rec_off", "file", "key_len", "value_pos", "value_size", "crc", "ts", "flags", "crc_calc")


@pytest.fixture(scope="module")
def g():
    import __graft_entry__

    __graft_entry__.build()
    import gocask_amd

    assert gocask_amd.device_count() > 0, "no GPU visible"
    return gocask_amd


def assert_same(got, gst, want, wst):
    assert gst["status"] == wst["status"], (gst, wst)
    if wst["status"]:
        assert gst["err_off"] == wst["err_off"] and gst["err_file"] == wst["err_file"]
    assert gst["final_last_offset"] == wst["final_last_offset"]
    assert len(got) == len(want), (len(got), len(want))
    for f in FIELDS:
        if not np.array_equal(got[f], want[f]):
            bad = np.nonzero(got[f] != want[f])[0][:5]
            raise AssertionError(f"field {f} differs at {bad}: got {got[f][bad]} want {want[f][bad]}")


def walk_sorted(files, names):
    walk = sorted(range(len(files)), key=lambda i: names[i])
    wf = [files[i] for i in walk]
    reset = [i + 1 < len(wf) for i in range(len(wf))]  # the lexically last file is active
    return wf, reset


# ------------------------------------------------------------------ golden ---
@pytest.mark.parametrize("name", case_names())
def test_golden_cases(g, orc, name):
    meta, files, reset = load_case(name)
    got, gst = g.replay(files, reset)
    check_case(meta, files, got, g.keydir(files, got), gst)
    want, wst = orc.replay(files, reset)
    assert_same(got, gst, want, wst)


@pytest.mark.parametrize("chunk", [4096, 1 << 16])
@pytest.mark.parametrize("name", ["datatxt_1000_puts", "existing_after_startup", "partial_write_desync"])
def test_golden_small_chunks(g, orc, name, chunk):
    meta, files, reset = load_case(name)
    got, gst = g.replay(files, reset, chunk_bytes=chunk, chunk_cap=8)
    want, wst = orc.replay(files, reset)
    assert_same(got, gst, want, wst)


# -------------------------------------------------------- NewDB / Open API ---
def test_newdb_in_memory_deleted_key(g):
    # core/db_test.go:375-393: Put foo, Delete foo, re-open -> ErrKeyNotFound
    data = orc_mod.entry(12345, b"foo", b"bar") + orc_mod.tombstone(12345, b"foo")
    db, err = g.NewDB("", g.NewInMemory(data))
    assert err is None
    v, err = db.Get(b"foo")
    assert err is g.ErrKeyNotFound and v is None
    assert db.Keys() == []
    assert db.last_offset == 41


def test_newdb_in_memory_datatxt(g):
    meta, files, reset = load_case("datatxt_1000_puts")
    db, err = g.NewDB("", g.NewInMemory(files[0].tobytes()))
    assert err is None
    assert sorted(db.Keys()) == sorted(meta["expect"])
    for k, e in meta["expect"].items():
        v, err = db.Get(k.encode())
        assert err is None and v == e["value"].encode()
    _, err = db.Get(b"")
    assert err is g.ErrInvalidKey


def test_newdb_crc_failed(g):
    meta, files, reset = load_case("crc_fail")
    db, err = g.NewDB("", g.NewInMemory(files[0].tobytes()))
    assert err is None
    v, err = db.Get(b"foo")
    assert err is g.ErrCRCFailed and v is None


def test_newdb_startup_error(g):
    meta, files, reset = load_case("partial_write_desync")
    db, err = g.NewDB("", g.NewInMemory(files[0].tobytes()))
    assert isinstance(err, g.StartupError) and str(err) == "gocask: startup error: unexpected EOF"
    assert db is not None and sorted(db.Keys()) == ["key", "user"]


def test_open_disk_lexical_walk_and_active_file(g, orc, tmp_path):
    # data_<n>_<unix>.csk names, 12 files, lexical walk + foo.txt skipped
    files, names = orc.gen_corpus(seed=21, val_fixed=0, key_min=8, key_max=12, key_universe=500,
                                  tomb_permille=30, max_file_size=1 << 16, n_files=12)
    d = tmp_path / "mydb"
    d.mkdir()
    for f, n in zip(files, names):
        (d / (n + ".csk")).write_bytes(f.tobytes())
    (d / "foo.txt").write_bytes(b"not a data file")
    db, err = g.Open("mydb", g.WithDataDir(str(tmp_path)))
    assert err is None
    assert db.active_file == "foo"  # lexically last entry of any kind (internal/fs/disk.go:56-67)
    assert db.files() == sorted(names)
    wf, _ = walk_sorted(files, names)
    want, wst = orc.replay(wf, [True] * len(wf))  # active "foo" never matches: always reset
    kd = orc.keydir(wf, want, [True] * len(wf))
    assert sorted(k.encode("utf-8", "surrogateescape") for k in db.Keys()) == sorted(kd)
    for k, r in list(kd.items())[:200]:
        e = db.Entry(k)
        assert e["ValuePos"] == int(r["value_pos"]) and e["CRC"] == int(r["crc"])
        assert e["File"] == sorted(names)[int(r["file"])]
        v, err = db.Get(k)
        assert err is None and zlib.crc32(v) == int(r["crc"])
    assert db.last_offset == wst["final_last_offset"]


def test_open_creates_active_file(g, tmp_path):
    db, err = g.Open("fresh", g.WithDataDir(str(tmp_path)))
    assert err is None and db.Keys() == []
    made = os.listdir(tmp_path / "fresh")
    assert len(made) == 1 and made[0].startswith("data_0_") and made[0].endswith(".csk")


# ------------------------------------------------------- device encoder (f4) --
@pytest.mark.parametrize("kw", [
    dict(seed=31, val_fixed=0, key_min=8, key_max=24, key_universe=1000, tomb_permille=10, flip_permille=10,
         max_file_size=1 << 20, n_files=5),
    dict(seed=32, val_fixed=1024, key_min=16, key_max=16, max_file_size=1 << 20, n_files=1),
])
def test_device_encoder_matches_oracle_generator(g, orc, kw):
    files, names = orc.gen_corpus(**kw)
    with g.ReplayContext() as ctx:
        info = ctx.encode(**kw)
        assert info["n_files"] == len(files)
        assert list(info["sizes"]) == [len(f) for f in files]
        for w, n in enumerate(info["walk_order"]):
            got = ctx.read_file(w, 0, len(files[n]))
            assert np.array_equal(got, files[n]), names[n]


# ------------------------------------------------------ randomised parity ---
CORPORA = [
    dict(seed=41, val_fixed=0, key_min=8, key_max=24, key_universe=2000, tomb_permille=10, flip_permille=10,
         max_file_size=4 << 20, n_files=4),
    dict(seed=42, val_fixed=100, key_min=8, key_max=8, key_universe=50, tomb_permille=200, max_file_size=1 << 18,
         n_files=6),
    dict(seed=43, val_fixed=4096, key_min=16, key_max=16, max_file_size=8 << 20, n_files=2),
]


@pytest.mark.parametrize("chunk,cap", [(4096, 2), (1 << 15, 256), (1 << 18, 256)])
@pytest.mark.parametrize("ci", range(len(CORPORA)))
def test_random_corpora(g, orc, ci, chunk, cap):
    files, names = orc.gen_corpus(**CORPORA[ci])
    wf, reset = walk_sorted(files, names)
    want, wst = orc.replay(wf, reset)
    got, gst = g.replay(wf, reset, chunk_bytes=chunk, chunk_cap=cap)
    assert_same(got, gst, want, wst)
    assert np.array_equal(got["flags"] & 2 == 0, want["crc_calc"] != want["crc"])


# ------------------------------------------------- multi-file runs, reruns ---
def test_multi_file_context(g, orc):
    # 12 rotated files (walk order != creation order) through a context
    kw = dict(seed=44, val_fixed=0, key_min=8, key_max=24, key_universe=20000, tomb_permille=10,
              flip_permille=10, max_file_size=6 << 20, n_files=12)
    files, names = orc.gen_corpus(**kw)
    wf, reset = walk_sorted(files, names)
    want, wst = orc.replay(wf, reset)
    with g.ReplayContext() as ctx:
        ctx.load(wf, reset)
        ctx.run()
        got, gst = ctx.fetch()
    assert_same(got, gst, want, wst)


def test_repeated_runs_identical_c3_shape(g):
    # C3 shape at 1/8 scale, device-encoded: back-to-back runs on one context
    # (capacities and the block queue reused) give identical tuples
    kw = dict(seed=3, val_fixed=0, key_min=8, key_max=24, key_universe=600000, tomb_permille=10,
              flip_permille=10, max_file_size=256 << 20, n_files=16)
    with g.ReplayContext() as ctx:
        ctx.encode(**kw)
        ctx.run()
        a, ast = ctx.fetch()
        for _ in range(3):
            ctx.run()
        b, bst = ctx.fetch()
    assert_same(a, ast, b, bst)
    assert ast["n_crc_fail"] > 0


def test_stage_overflow_rewalks(g, orc):
    # 20-byte records with a 16-record stage: chunks overflow their stage and
    # k_compact re-walks them straight into the record table
    recs = [orc_mod.entry(i, b"k%d" % (i % 7), b"") for i in range(4000)]
    files = [b"".join(recs[:2000]), b"".join(recs[2000:])]
    reset = [True, False]
    want, wst = orc.replay(files, reset)
    with g.ReplayContext(chunk_bytes=4096, chunk_cap=16) as ctx:
        ctx.load(files, reset)
        ctx.run()
        got, gst = ctx.fetch()
        st = ctx.stats()
    assert st["n_overflow"] >= 1
    assert_same(got, gst, want, wst)


# ---------------------------------- second run: no host round trip (device) ---
def _run_twice(g, files, reset, **kw):
    with g.ReplayContext(**kw) as ctx:
        ctx.load(files, reset)
        ctx.run()
        first = ctx.fetch()
        ctx.run()
        second = ctx.fetch()
        st = ctx.stats()
    return first, second, st


@pytest.mark.parametrize("name", case_names())
def test_golden_cases_device_path(g, orc, name):
    # the second run of a context takes the device-only path (EOF verdicts,
    # carries and the record count on the device): same answers as the oracle
    meta, files, reset = load_case(name)
    want, wst = orc.replay(files, reset)
    (a, ast), (b, bst), st = _run_twice(g, files, reset)
    assert_same(a, ast, want, wst)
    assert_same(b, bst, want, wst)
    if len(want):
        assert st["device_path"] and st["n_reruns"] == 0


def test_eof_classes_device_path(g, orc):
    base = b"".join(orc_mod.entry(i, b"key%04d" % i, b"v" * (i % 97)) for i in range(300))
    tails = [b"", b"\x01" * 9, struct.pack("<IIII", 0, 1, 5, 5) + b"ab", orc_mod.entry(1, b"kk", b"value")[:-2]]
    for t in tails:
        files = [base, t, base]
        reset = [True, False, True]
        want, wst = orc.replay(files, reset)
        (a, ast), (b, bst), st = _run_twice(g, files, reset, chunk_bytes=4096)
        assert_same(b, bst, want, wst)
        assert st["device_path"]


def test_device_path_capacity_rerun(g, orc):
    # a context sized by a small corpus, then loaded with a larger one: the
    # device-only run exceeds the record-table capacity and is redone on the
    # host path, exactly
    small = [b"".join(orc_mod.entry(i, b"k%d" % i, b"x" * 40) for i in range(100))]
    big = [b"".join(orc_mod.entry(i, b"k%d" % i, b"y" * 30) for i in range(5000))]
    want, wst = orc.replay(big, [True])
    with g.ReplayContext(chunk_bytes=4096) as ctx:
        ctx.load(small, [True])
        ctx.run()
        ctx.load(big, [True])
        ctx.run()
        got, gst = ctx.fetch()
        st = ctx.stats()
    assert st["n_reruns"] >= 1 and not st["device_path"]
    assert_same(got, gst, want, wst)


# ---------------------------------------------- device keydir (row f1) ---
def _expected_keydir(files, want, keep_tombstones=False):
    """Apply the oracle's records in walk order (core/keydir.go:22-49):
    {key: record}; with keep_tombstones, the last record of every key."""
    kd = {}
    for r in want:
        o = int(r["rec_off"]) + 16
        key = bytes(files[int(r["file"])][o:o + int(r["key_len"])])
        if int(r["flags"]) & 1 and not keep_tombstones:
            kd.pop(key, None)
        else:
            kd.pop(key, None)  # re-insert: dict order = walk order of the winners
            kd[key] = r
    return kd


def _check_keydir(files, got, kd):
    assert len(got) == len(kd), (len(got), len(kd))
    win = sorted(kd.values(), key=lambda r: (int(r["file"]), int(r["rec_off"])))
    for a, b in zip(got, win):  # walk order of the winning records
        for f in FIELDS:
            assert a[f] == b[f], (f, a, b)


@pytest.mark.parametrize("name", case_names())
def test_keydir_golden(g, orc, name):
    meta, files, reset = load_case(name)
    want, wst = orc.replay(files, reset)
    with g.ReplayContext() as ctx:
        ctx.load(files, reset)
        ctx.run()
        live, _ = ctx.keydir()
        every, _ = ctx.keydir(keep_tombstones=True)
    _check_keydir(files, live, _expected_keydir(files, want))
    _check_keydir(files, every, _expected_keydir(files, want, keep_tombstones=True))
    # the reference's own known answers: the live keys of the fixture
    if meta["status"] != "unexpected_eof":
        keys = {bytes(files[int(r["file"])][int(r["rec_off"]) + 16:int(r["rec_off"]) + 16 + int(r["key_len"])])
                for r in live}
        assert keys == {k.encode() for k in meta["expect"]}


@pytest.mark.parametrize("ci", range(len(CORPORA)))
def test_keydir_random(g, orc, ci):
    files, names = orc.gen_corpus(**CORPORA[ci])
    wf, reset = walk_sorted(files, names)
    want, wst = orc.replay(wf, reset)
    with g.ReplayContext() as ctx:
        ctx.load(wf, reset)
        ctx.run()
        live, _ = ctx.keydir()
        every, _ = ctx.keydir(keep_tombstones=True)
    _check_keydir(wf, live, _expected_keydir(wf, want))
    _check_keydir(wf, every, _expected_keydir(wf, want, keep_tombstones=True))


def test_keydir_c3_shape_device_encoded(g):
    # C3 shape at 1/64 scale (16 rotated files, Zipf values, 1 % tombstones,
    # a key universe of half the records): files read back from the device
    kw = dict(seed=3, val_fixed=0, key_min=8, key_max=24, key_universe=80000, tomb_permille=10,
              flip_permille=10, max_file_size=32 << 20, n_files=16)
    with g.ReplayContext() as ctx:
        info = ctx.encode(**kw)
        ctx.run()
        recs, st = ctx.fetch()
        files = [ctx.read_file(w, 0, int(info["sizes"][info["walk_order"][w]])) for w in range(info["n_files"])]
        live, ms = ctx.keydir()
    assert st["status"] == 0 and len(recs) > 100000
    _check_keydir(files, live, _expected_keydir(files, recs))


def test_pinned_host_load_and_fetch_into(g, orc):
    # the host-inclusive path of bench.py: files in registered (pinned) host
    # memory, tuples copied into a registered REC_DTYPE array
    kw = dict(seed=45, val_fixed=0, key_min=8, key_max=24, key_universe=5000, tomb_permille=10,
              flip_permille=10, max_file_size=2 << 20, n_files=3)
    files, names = orc.gen_corpus(**kw)
    wf, reset = walk_sorted(files, names)
    want, wst = orc.replay(wf, reset)
    host = np.concatenate([np.frombuffer(f, np.uint8) for f in wf])
    g.host_register(host)
    views, off = [], 0
    for f in wf:
        views.append(host[off:off + len(f)])
        off += len(f)
    recs = np.zeros(len(want) + 5, dtype=g.REC_DTYPE)
    g.host_register(recs)
    try:
        with g.ReplayContext() as ctx:
            ctx.load(views, reset)
            ctx.run()
            n = ctx.fetch_into(recs)
            _, gst = ctx.fetch()
    finally:
        g.host_unregister(host)
        g.host_unregister(recs)
    assert n == len(want)
    assert_same(recs[:n], gst, want, wst)


def test_tiny_records_and_empty_values(g, orc):
    rng = np.random.default_rng(7)
    recs = []
    for i in range(3000):
        k = bytes(rng.integers(0, 256, int(rng.integers(1, 4)), dtype=np.uint8))
        r = int(rng.integers(0, 10))
        if r == 0:
            recs.append(orc_mod.tombstone(i, k))
        elif r == 1:
            recs.append(orc_mod.entry(i, k, b""))
        else:
            recs.append(orc_mod.entry(i, k, bytes(rng.integers(0, 256, int(rng.integers(1, 40)), dtype=np.uint8))))
    data = b"".join(recs)
    for chunk in (4096, 1 << 16):
        want, wst = orc.replay([data], [False])
        got, gst = g.replay([data], [False], chunk_bytes=chunk, chunk_cap=16)
        assert_same(got, gst, want, wst)


def test_values_that_look_like_records(g, orc):
    # values that are themselves serialized records: speculation will land inside
    # them; validation + fixup must still produce the reference's chain
    rng = np.random.default_rng(9)
    parts = []
    for i in range(400):
        inner = b"".join(orc_mod.entry(j, b"inner%d" % j, bytes(rng.integers(0, 256, 300, dtype=np.uint8)))
                         for j in range(int(rng.integers(1, 30))))
        parts.append(orc_mod.entry(i, b"outer%05d" % i, inner))
    data = b"".join(parts)
    want, wst = orc.replay([data], [True])
    for chunk in (4096, 1 << 14):
        got, gst = g.replay([data], [True], chunk_bytes=chunk)
        assert_same(got, gst, want, wst)


def test_eof_classes_at_every_chunk_phase(g, orc):
    base = b"".join(orc_mod.entry(i, b"key%04d" % i, b"v" * (i % 97)) for i in range(300))
    tails = [b"", b"\x01" * 9, struct.pack("<IIII", 0, 1, 5, 5), struct.pack("<IIII", 0, 1, 5, 5) + b"ab",
             orc_mod.entry(1, b"kk", b"value")[:-2]]
    for cut in (0, 1, 17, 4000):
        for t in tails:
            files = [base[:len(base) - cut] if cut else base, t + b"", base]
            reset = [True, False, True]
            want, wst = orc.replay(files, reset)
            got, gst = g.replay(files, reset, chunk_bytes=4096)
            assert_same(got, gst, want, wst)


# ------------------------------------------------------------ config sizes ---
def test_config1_64mib_vs_oracle(g, orc):
    kw = dict(seed=1, val_fixed=1024, key_min=16, key_max=16, max_file_size=64 << 20, n_files=1)
    files, names = orc.gen_corpus(**kw)
    assert len(files[0]) == 67108800
    want, wst = orc.replay(files, [False])
    with g.ReplayContext() as ctx:
        ctx.encode(**kw)
        ctx.run()
        got, gst = ctx.fetch()
    assert_same(got, gst, want, wst)
    assert len(got) == 63550


def test_config2_8gib_value_pos_wraps(g):
    # 1 x 8 GiB, 4 KiB values: ValuePos is uint32 and wraps (core/keydir.go:25)
    kw = dict(seed=2, val_fixed=4096, key_min=16, key_max=16, max_file_size=8 << 30, n_files=1)
    with g.ReplayContext() as ctx:
        info = ctx.encode(**kw)
        assert info["n_ops"] == 2080895 and int(info["sizes"][0]) == 8589934560
        ctx.run()
        got, gst = ctx.fetch()
        st = ctx.stats()
        # independent of the device: ~2,000 records spread over the file, half
        # of them past the 4 GiB wrap, read back from the resident bytes; the
        # header by struct.unpack (core/header.go:58-62), the verdict by
        # zlib.crc32 of the value (= Go's crc32.ChecksumIEEE)
        rng = np.random.default_rng(8)
        wrap = (1 << 32) // 4128
        picks = np.concatenate([rng.choice(wrap, 1000, replace=False),
                                wrap + 1 + rng.choice(len(got) - wrap - 1, 1000, replace=False), [0, len(got) - 1]])
        for r in picks.tolist():
            rec = got[r]
            raw = bytes(ctx.read_file(0, int(rec["rec_off"]), 4128))
            crc, ts, ks, vs = struct.unpack("<IIII", raw[:16])
            assert (crc, ts, ks, vs) == (int(rec["crc"]), int(rec["ts"]), int(rec["key_len"]), int(rec["value_size"]))
            assert zlib.crc32(raw[32:]) == crc == int(rec["crc_calc"]), r
            assert int(rec["value_pos"]) == (int(rec["rec_off"]) + 32) % (1 << 32)
    assert (picks >= wrap).sum() >= 1000
    assert gst["status"] == 0 and len(got) == 2080895 and st["n_crc_fail"] == 0
    i = np.arange(len(got), dtype=np.uint64)
    assert np.array_equal(got["rec_off"], i * np.uint64(4128))
    assert np.array_equal(got["value_pos"], ((i * np.uint64(4128) + np.uint64(32)) % np.uint64(1 << 32)).astype(np.uint32))
    assert (got["flags"] & 2).all()
    assert np.array_equal(got["ts"], (np.uint64(1700000000) + i).astype(np.uint32))


def test_config5_bitflips_reject_set(g):
    # C5 shape at 1/8 scale (4 GiB): rejects must be exactly the flipped records
    import spec

    kw = dict(seed=5, val_fixed=0, key_min=8, key_max=24, key_universe=600000, tomb_permille=10,
              flip_permille=10, max_file_size=2 << 30, n_files=2)
    with g.ReplayContext() as ctx:
        ctx.encode(**kw)
        ctx.run()
        got, gst = ctx.fetch()
    assert gst["status"] == 0 and len(got) > 100000
    ops = (got["ts"].astype(np.uint64) - np.uint64(1700000000)) % np.uint64(1 << 32)
    flipped = spec.expected_flips(5, ops, 10, 10)
    rejected = (got["flags"] & 2) == 0
    assert flipped.sum() > 1000
    assert np.array_equal(rejected, flipped)
    tomb = (got["flags"] & 1) == 1
    assert np.array_equal(tomb, (spec.H(5, 3, ops) % np.uint64(1000)) < np.uint64(10))


def test_keys_longer_than_speculation_bound(g, orc):
    # keys of 64 KiB and more are never speculated (the prefilter needs
    # KeySize <= 65535): chunks whose only headers carry such keys get a
    # wrong or no entry and validation + fixup must recover the chain; also a
    # tombstone whose "key" is that long and values past 64 KiB
    rng = np.random.default_rng(11)

    def rb(n):
        return bytes(rng.integers(0, 256, n, dtype=np.uint8))

    parts = []
    for i in range(60):
        r = i % 6
        if r == 0:
            parts.append(orc_mod.entry(i, b"big%02d" % i + rb(70000 + 997 * i), rb(int(rng.integers(0, 300)))))
        elif r == 1:
            parts.append(orc_mod.tombstone(i, b"tomb%02d" % i + rb(66000 + 13 * i)))
        elif r == 2:
            parts.append(orc_mod.entry(i, b"k%03d" % i, rb(200000 + 31 * i)))
        else:
            parts.append(orc_mod.entry(i, b"k%03d" % i, rb(int(rng.integers(1, 5000)))))
    data = b"".join(parts)
    want, wst = orc.replay([data], [False])
    for chunk, mk in ((4096, 0), (1 << 16, 0), (1 << 16, 1024)):
        got, gst = g.replay([data], [False], chunk_bytes=chunk, **({"max_key": mk} if mk else {}))
        assert_same(got, gst, want, wst)
    with g.ReplayContext(chunk_bytes=4096) as ctx:  # keydir and Get of the long keys
        ctx.load([data], [False])
        ctx.run()
        live, _ = ctx.keydir()
        keys = [bytes(data[int(r["rec_off"]) + 16:int(r["rec_off"]) + 16 + int(r["key_len"])]) for r in live]
        st, vs, cc, vals = ctx.get_batch(keys)
    assert len(live) == 50 and all(s == 0 for s in st)
    assert max(len(k) for k in keys) > 65535


# ------------------------------------- pipelined host-in/host-out replay ---
@pytest.mark.parametrize("fsize", [200 << 20, (215 << 20) + (100 << 10)])
def test_replay_grouped_equals_oracle(g, orc, monkeypatch, fsize):
    # gck_replay / gck_replay_into cut the files into >= 1 GiB groups after
    # files that reset lastOffset; with 12 x ~200 MiB files and the active
    # file in the middle, groups must neither split a carry nor reorder.
    # (~215.1 MiB files: 431 chunks each, so a later group's first chunk is
    # not a multiple of 4 and k_scan_local takes its unaligned path)
    kw = dict(seed=46, val_fixed=0, key_min=8, key_max=24, key_universe=200000, tomb_permille=10,
              flip_permille=10, max_file_size=fsize, n_files=12)
    files, names = orc.gen_corpus(**kw)
    wf, _ = walk_sorted(files, names)
    reset = [True] * len(wf)
    reset[5] = False  # the active file walked mid-way: lastOffset carries into file 6
    want, wst = orc.replay(wf, reset)
    got, gst = g.replay(wf, reset)
    assert_same(got, gst, want, wst)
    recs = np.zeros(len(want) + 3, dtype=g.REC_DTYPE)
    st = g.replay_into(wf, recs, reset)
    assert_same(recs[:st["n_recs"]], st, want, wst)
    small = np.zeros(10, dtype=g.REC_DTYPE)
    with pytest.raises(Exception):
        g.replay_into(wf, small, reset)
    # the contexts kept from the calls above serve the next ones (same answers),
    # and after gck_replay_release_cache new ones do
    # (a pinned array: the tuples are written by k_push_recs over PCIe)
    recs2 = np.zeros(len(want), dtype=g.REC_DTYPE)
    g.host_register(recs2)
    try:
        st2 = g.replay_into(wf, recs2, reset)
        assert_same(recs2[:st2["n_recs"]], st2, want, wst)
    finally:
        g.host_unregister(recs2)
    g.release_cache()
    got3, gst3 = g.replay(wf, reset)
    assert_same(got3, gst3, want, wst)


def test_replay_grouped_startup_error(g, orc):
    # a startup error in a later group: the records before it, nothing after
    big = [orc.gen_corpus(seed=47 + i, val_fixed=4096, key_min=16, key_max=16, max_file_size=600 << 20,
                          n_files=1)[0][0] for i in range(3)]
    bad = np.frombuffer(orc_mod.entry(1, b"user", b"x" * 10) + orc_mod.entry(2, b"key", b"yy")[:-4], np.uint8)
    wf = [big[0], big[1], bad, big[2]]
    reset = [True, True, True, False]
    want, wst = orc.replay(wf, reset)
    assert wst["status"] == 1 and wst["err_file"] == 2
    got, gst = g.replay(wf, reset)
    assert_same(got, gst, want, wst)
    assert gst["files_walked"] == wst["files_walked"] == 3
