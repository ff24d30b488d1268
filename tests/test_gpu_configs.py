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


def test_config4_last_rank_shard_16x2gib(g, orc):
    """BASELINE C4 at full size on one GPU: the shard bench.py's rank 7 replays
    at N = 8 (16 x 2 GiB of the 128-file corpus, its last file the active one),
    with the corpus-wide key universe (keys repeat across files: the keydir is
    built across files, core/keydir.go:22-49).  Checked by the spec's
    properties (as C3, per file; key lengths from the shared key ids), the
    active file against the oracle field for field, and the keydir merge over a
    one-rank RCCL group against the last writer of every key id."""
    import socket

    import torch
    import torch.distributed as dist

    from gocask_amd import shard

    world, rank = 8, 7
    ids, last_active, kw = bench.c4_spec(world, rank)
    assert last_active and len(ids) == 16 and kw["key_seed"] == 4
    U = kw["key_universe"]
    assert U == 312_500 * 128
    base = rank * 16  # the files of lower ranks (shard.file_base at N = 8)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        with g.ReplayContext() as ctx:
            info = ctx.encode_files(ids, last_is_active=True, **kw)
            ctx.run()
            got, st = ctx.fetch()
            stats = ctx.stats()
            n_live, ph = shard.merge_keydir(ctx, dist, base)
            ents, _ = ctx.kd_fetch_merged()
    finally:
        dist.destroy_process_group()
    nf = len(ids)
    sizes = [int(x) for x in info["sizes"]]
    assert sum(sizes) > 31 << 30
    assert st["status"] == 0 and len(got) == info["n_ops"] and stats["n_crc_fail"] == 0
    assert st["final_last_offset"] == sizes[-1] % (1 << 32)  # the active file does not reset
    fidx = got["file"].astype(np.int64)
    assert (np.diff(fidx) >= 0).all() and fidx[0] == 0 and fidx[-1] == nf - 1
    tomb = (got["flags"] & 1) == 1
    off = got["rec_off"].astype(np.uint64)
    klen = got["key_len"].astype(np.uint64)
    vsz = got["value_size"].astype(np.uint64)
    ent = np.uint64(16) + klen + np.where(tomb, np.uint64(0), vsz)
    ks = np.where(tomb, np.uint64(0), klen)
    assert np.array_equal(got["value_pos"], ((off + np.uint64(16) + ks) % np.uint64(1 << 32)).astype(np.uint32))
    assert ((got["flags"] & 2) == 2).all() and np.array_equal(got["crc_calc"], got["crc"])
    bounds = np.searchsorted(fidx, np.arange(nf + 1))
    keyid = np.zeros(len(got), dtype=np.uint64)
    for w, n in enumerate(ids):
        a, b = bounds[w], bounds[w + 1]
        assert b > a and off[a] == 0
        assert np.array_equal(off[a + 1:b], off[a:b - 1] + ent[a:b - 1]), w
        assert int(off[b - 1] + ent[b - 1]) == sizes[w], w
        ops = got["ts"][a:b].astype(np.uint64) - np.uint64(TS0)
        assert np.array_equal(ops, np.arange(b - a, dtype=np.uint64)), w  # op i of the file, in order
        assert np.array_equal(tomb[a:b], (spec.H(4 + n, 3, ops) % np.uint64(1000)) < np.uint64(kw["tomb_permille"]))
        # keys from the corpus-wide universe: op i of file n draws key id
        # H(4, 1, n << 32 | i) % U, its length key_min + H(4, 6, id) % 17
        keyid[a:b] = spec.H(4, 1, (np.uint64(n) << np.uint64(32)) | ops) % np.uint64(U)
    want_len = np.uint64(kw["key_min"]) + spec.H(4, 6, keyid) % np.uint64(kw["key_max"] - kw["key_min"] + 1)
    assert np.array_equal(klen, want_len)
    # keys repeat across the shard's files
    first = np.unique(keyid, return_index=True)[1]
    last_rev = np.unique(keyid[::-1], return_index=True)[1]
    last = len(keyid) - 1 - last_rev
    assert (fidx[last] != fidx[first]).sum() > 100_000
    # the merged keydir = the last record of every key id, kept if a Put
    live = last[~tomb[last]]
    assert n_live == len(ents) == len(live)
    got_pairs = np.sort(ents["rec"]["file"].astype(np.uint64) << np.uint64(40) | ents["rec"]["rec_off"].astype(np.uint64))
    want_pairs = np.sort((fidx[live].astype(np.uint64) + np.uint64(base)) << np.uint64(40) | off[live])
    assert np.array_equal(got_pairs, want_pairs)
    assert ph["status"]["status"] == 0
    # the active file (2 GiB) against the oracle, field for field
    n = ids[-1]
    files, _ = orc.gen_corpus(**{**kw, "seed": 4 + n, "key_file": n})
    assert len(files[0]) == sizes[-1]
    want, wst = orc.replay(files, [False])
    a = bounds[nf - 1]
    assert wst["status"] == 0 and len(want) == len(got) - a
    for f in FIELDS:
        w = want[f] + (nf - 1 if f == "file" else 0)
        assert np.array_equal(got[f][a:], w), f
