"""Corruption fuzz parity (GPU box): seeded corpora with 1-3 random bit flips
anywhere -- headers and keys included, not only values -- replayed through the
C-ABI and compared with the oracle record for record, with the same status,
error file / offset, files walked and final lastOffset.

A flipped KeySize / ValueSize desynchronises the reader
(core/db.go:145-178): huge sizes end a file silently (bufio.Reader.Discard's
io.EOF) or with "unexpected EOF" (a partial header or key, io.ReadFull), and
the bytes after a desync are read as headers (core/header.go:58-62).  The
device's speculation, validation and fix-up must reach exactly the reference's
answer wherever that happens ("header flips are a separate
error-parity test").
"""
import numpy as np
import pytest

import bench

FIELDS = ("rec_off", "file", "key_len", "value_pos", "value_size", "crc", "ts", "flags", "crc_calc")
N_CORPORA = 240
BATCH = 20


@pytest.fixture(scope="module")
def g():
    import __graft_entry__

    __graft_entry__.build()
    import gocask_amd

    assert gocask_amd.device_count() > 0, "no GPU visible"
    return gocask_amd


def _same(got, gst, want, wst, what):
    for k in ("status", "err_file", "err_off", "files_walked", "final_last_offset"):
        if k in ("err_file", "err_off") and not wst["status"]:
            continue
        assert gst[k] == wst[k], (what, k, gst, wst)
    assert len(got) == len(want), (what, len(got), len(want))
    for f in FIELDS:
        if not np.array_equal(got[f], want[f]):
            bad = np.nonzero(got[f] != want[f])[0][:5]
            raise AssertionError(f"{what}: field {f} differs at {bad}: got {got[f][bad]} want {want[f][bad]}")


def _flip(orc, rng, wf, reset, nflip, header_share=0.6):
    """Flip nflip random bits: header or key bytes of a random record of the
    clean corpus (share header_share), else any byte of any file."""
    clean, _ = orc.replay(wf, reset)
    wf = [f.copy() for f in wf]
    where = []
    for _ in range(nflip):
        if len(clean) and rng.random() < header_share:
            r = clean[int(rng.integers(len(clean)))]
            f = int(r["file"])
            pos = int(r["rec_off"]) + int(rng.integers(16 + int(r["key_len"])))
        else:
            f = int(rng.integers(len(wf)))
            if not len(wf[f]):
                continue
            pos = int(rng.integers(len(wf[f])))
        bit = int(rng.integers(8))
        wf[f][pos] ^= np.uint8(1 << bit)
        where.append((f, pos, bit))
    return wf, where


def _corpus(orc, seed):
    rng = np.random.default_rng(seed)
    kind = seed % 4
    if kind == 0:  # Zipf values, updates and deletes
        kw = dict(val_fixed=0, key_min=8, key_max=24, key_universe=200, tomb_permille=50,
                  max_file_size=int(rng.integers(16 << 10, 256 << 10)), n_files=3)
    elif kind == 1:  # many small records
        kw = dict(val_fixed=int(rng.integers(1, 100)), key_min=8, key_max=40, key_universe=300, tomb_permille=100,
                  max_file_size=int(rng.integers(8 << 10, 64 << 10)), n_files=4)
    elif kind == 2:  # long keys
        kw = dict(val_fixed=0, key_min=8, key_max=512, key_universe=100, tomb_permille=30,
                  max_file_size=int(rng.integers(32 << 10, 128 << 10)), n_files=2)
    else:  # tiny records: several per 16 B block of the CRC pass
        kw = dict(val_fixed=int(rng.integers(0, 8)), key_min=8, key_max=9, key_universe=50, tomb_permille=200,
                  max_file_size=int(rng.integers(4 << 10, 16 << 10)), n_files=3)
    files, names = orc.gen_corpus(seed=1000 + seed, **kw)
    walk = sorted(range(len(files)), key=lambda i: names[i])
    wf = [files[i] for i in walk]
    reset = [i + 1 < len(wf) for i in range(len(wf))]
    wf, where = _flip(orc, rng, wf, reset, int(rng.integers(1, 4)))
    return wf, reset, where


@pytest.mark.gpu
@pytest.mark.parametrize("b0", range(0, N_CORPORA, BATCH))
def test_bit_flips_anywhere(g, orc, b0):
    """Both chunk sizes on gck_replay (pooled contexts, the device-only run
    path), and the host run path then the device-only path of one context."""
    statuses = set()
    for seed in range(b0, b0 + BATCH):
        wf, reset, where = _corpus(orc, seed)
        want, wst = orc.replay(wf, reset)
        statuses.add(wst["status"])
        for chunk in (4 << 10, 512 << 10):
            got, gst = g.replay(wf, reset, chunk_bytes=chunk)
            _same(got, gst, want, wst, f"seed {seed} chunk {chunk} flips {where}")
        with g.ReplayContext(chunk_bytes=4 << 10) as ctx:
            ctx.load(wf, reset)
            for run in range(2):
                ctx.run()
                got, gst = ctx.fetch()
                _same(got, gst, want, wst, f"seed {seed} context run {run} flips {where}")
    assert statuses  # (startup errors and clean ends both occur over the batches)


def test_bit_flips_cover_the_error_classes(orc):
    """The fuzz corpora reach every outcome of the reference's reader: clean
    replays, silent truncation (records lost without an error), and startup
    errors (CPU: the oracle's view of the same corpora)."""
    outcomes = dict(error=0, truncated=0, clean=0)
    for seed in range(N_CORPORA):
        wf, reset, _ = _corpus(orc, seed)
        _, wst = orc.replay(wf, reset)
        ends = sum(len(f) for f in wf)
        if wst["status"]:
            outcomes["error"] += 1
        else:
            recs, _ = orc.replay(wf, reset)
            covered = sum(16 + int(r["key_len"]) + (0 if r["flags"] & 1 else int(r["value_size"])) for r in recs)
            outcomes["truncated" if covered < ends else "clean"] += 1
    assert all(v >= 10 for v in outcomes.values()), outcomes


@pytest.mark.gpu
def test_c3_file_with_100_header_flips(g, orc):
    """Walk file 0 of the C3 workload (2 GiB, 640 K records) with 100 random
    header bits flipped, against the oracle."""
    kw = dict(bench.CONFIGS["c3"], n_files=1)
    files, _ = orc.gen_corpus(**kw)
    f = files[0]
    clean, _ = orc.replay([f], [True])
    rng = np.random.default_rng(2024)
    for i in rng.choice(len(clean), 100, replace=False):
        f[int(clean[i]["rec_off"]) + int(rng.integers(16))] ^= np.uint8(1 << int(rng.integers(8)))
    want, wst = orc.replay([f], [True])
    # the records before the first desync are the clean ones (offsets agree);
    # past it the reference reads whatever the bytes say
    n = min(len(want), len(clean))
    diff = np.nonzero(want["rec_off"][:n] != clean["rec_off"][:n])[0]
    first = int(diff[0]) if len(diff) else n
    print(f"c3 file 0, 100 header flips: {len(want)} records replayed, {first} before the first desync, "
          f"{len(clean)} clean; status {wst['status']}")
    assert 0 < first <= len(want)
    with g.ReplayContext() as ctx:
        ctx.load([f], [True])
        for run in range(2):
            ctx.run()
            got, gst = ctx.fetch()
            _same(got, gst, want, wst, f"c3 file 0 run {run}")


@pytest.mark.gpu
def test_c3_file_1000_crc_and_timestamp_flips(g, orc):
    """Walk file 0 of C3 with 1,000 random bits flipped inside the CRC and
    Timestamp words of headers (core/header.go:9-16: bytes 0-7), which never
    desynchronise the reader: every record is still replayed, the reject set
    (core/db.go:311: ke.CRC != CalcCRC32(value)) is exactly the records whose
    CRC word was flipped, the flipped timestamps read back as struct.unpack
    of the flipped bytes, and everything else equals the oracle field for
    field."""
    import struct

    kw = dict(bench.CONFIGS["c3"], n_files=1)
    files, _ = orc.gen_corpus(**kw)
    f = files[0]
    clean, _ = orc.replay([f], [True])
    assert clean["flags"].min() & 2, "the C3 spec has no corrupt values"
    rng = np.random.default_rng(4242)
    picks = rng.choice(len(clean), 1000, replace=False)
    crc_hit, ts_hit = set(), set()
    for i in picks:
        o = int(clean[int(i)]["rec_off"])
        byte = int(rng.integers(8))  # 0-3 CRC, 4-7 Timestamp
        f[o + byte] ^= np.uint8(1 << int(rng.integers(8)))
        (crc_hit if byte < 4 else ts_hit).add(int(i))
    want, wst = orc.replay([f], [True])
    assert wst["status"] == 0 and len(want) == len(clean)
    assert np.array_equal(want["rec_off"], clean["rec_off"])
    rejects = set(np.nonzero((want["flags"] & 2) == 0)[0].tolist())
    assert rejects == crc_hit and len(crc_hit) > 400
    with g.ReplayContext() as ctx:
        ctx.load([f], [True])
        for run in range(2):
            ctx.run()
            got, gst = ctx.fetch()
            _same(got, gst, want, wst, f"c3 file 0 crc/ts flips run {run}")
            assert set(np.nonzero((got["flags"] & 2) == 0)[0].tolist()) == crc_hit
            fb = f.tobytes() if hasattr(f, "tobytes") else bytes(f)
            for i in sorted(ts_hit)[:200] + sorted(crc_hit)[:200]:
                o = int(got[i]["rec_off"])
                crc, ts = struct.unpack_from("<II", fb, o)
                assert int(got[i]["ts"]) == ts and int(got[i]["crc"]) == crc, i
    print(f"c3 file 0: {len(crc_hit)} CRC-word and {len(ts_hit)} timestamp-word flips, "
          f"{len(want)} records compared, reject set = CRC-flipped set")
