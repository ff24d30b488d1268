"""Keydir merge across shards on one GPU, through the C-ABI.

A corpus is cut into shards of consecutive files (walk order); every shard is
replayed by its own context, its keydir (tombstones kept) packed into nparts
partitions, each owner merges partition p of every shard in shard order.  The
owners' entries together must equal the keydir keyDir.set / unset builds over
the whole corpus in walk order (core/keydir.go:22-49), computed from the
oracle's records.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

FIELDS = ("rec_off", "file", "key_len", "value_pos", "value_size", "crc", "ts", "flags", "crc_calc")


@pytest.fixture(scope="module")
def g():
    import __graft_entry__

    __graft_entry__.build()
    import gocask_amd

    assert gocask_amd.device_count() > 0, "no GPU visible"
    return gocask_amd


def _walk(files, names):
    walk = sorted(range(len(files)), key=lambda i: names[i])
    wf = [files[i] for i in walk]
    return wf, [i + 1 < len(wf) for i in range(len(wf))]


def _global_keydir(files, recs):
    """{key: record} over all files in walk order, deletes applied."""
    kd = {}
    for r in recs:
        o = int(r["rec_off"]) + 16
        key = bytes(files[int(r["file"])][o:o + int(r["key_len"])])
        if int(r["flags"]) & 1:
            kd.pop(key, None)
        else:
            kd[key] = r
    return kd


def _pack_shards(g, torch, shards, nparts):
    """Replay every shard on its own context and pack its keydir."""
    out, base = [], 0
    for s, (files, reset) in enumerate(shards):
        ctx = g.ReplayContext()
        ctx.load(files, reset)
        ctx.run()
        ctx.keydir(keep_tombstones=True, fetch=False)
        counts, kb = ctx.kd_pack_sizes(nparts)
        ents = torch.empty(max(sum(counts) * 64, 1), dtype=torch.uint8, device="cuda")
        keys = torch.empty(max(sum(kb), 1), dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        ctx.kd_pack(s, base, ents.data_ptr(), sum(counts), keys.data_ptr(), sum(kb))
        out.append((ctx, ents, keys, counts, kb, len(files)))
        base += len(files)
    return out


def _merge_owner(torch, packed, p, owner_ctx):
    """Owner p: partition p of every shard, in shard order (what the
    all-to-all delivers), merged on owner_ctx."""
    e_parts, k_parts, cnts, kbs = [], [], [], []
    for _, ents, keys, counts, kb, _ in packed:
        eo, ko = sum(counts[:p]) * 64, sum(kb[:p])
        e_parts.append(ents[eo:eo + counts[p] * 64])
        k_parts.append(keys[ko:ko + kb[p]])
        cnts.append(counts[p])
        kbs.append(kb[p])
    pad = torch.zeros(8, dtype=torch.uint8, device="cuda")
    E = torch.cat(e_parts + [pad])
    K = torch.cat(k_parts + [pad])
    torch.cuda.synchronize()
    n, _ = owner_ctx.kd_merge(E.data_ptr(), K.data_ptr(), cnts, kbs)
    ents, keys = owner_ctx.kd_fetch_merged()
    assert len(ents) == n
    return ents, keys


def _check_merged(files, owners, want_kd, nparts, shard_of_file):
    seen = {}
    for p, (ents, keys) in enumerate(owners):
        if len(ents):
            assert np.all((ents["hash"] >> np.uint64(40)) % np.uint64(nparts) == np.uint64(p))
            order = list(zip(ents["rec"]["file"].tolist(), ents["rec"]["rec_off"].tolist()))
            assert order == sorted(order)  # shard order, then walk order
        for e in ents:
            ko, kl = int(e["key_off"]), int(e["key_len"])
            assert ko % 8 == 0
            key = bytes(keys[ko:ko + kl])
            assert not keys[ko + kl:ko + ((kl + 7) & ~7)].any()  # zero padding
            assert key not in seen, "key owned twice"
            seen[key] = e
    assert set(seen) == set(want_kd), (len(seen), len(want_kd))
    for key, e in seen.items():
        r = want_kd[key]
        for f in FIELDS:
            assert e["rec"][f] == r[f], (key, f, e["rec"][f], r[f])
        assert e["key_len"] == r["key_len"] and e["shard"] == shard_of_file[int(r["file"])]
        o = int(r["rec_off"]) + 16
        assert key == bytes(files[int(r["file"])][o:o + int(r["key_len"])])


@pytest.mark.parametrize("cuts,nparts", [((2, 4), 1), ((2, 4), 3), ((1, 3, 5), 4), ((3,), 8), ((), 2)])
def test_merge_shards_equals_global_keydir(g, orc, cuts, nparts):
    import torch

    # a small key universe and 20 % deletes: keys cross shards, deletes in a
    # later shard must hide Puts of an earlier one
    files, names = orc.gen_corpus(seed=71, val_fixed=0, key_min=8, key_max=24, key_universe=1500,
                                  tomb_permille=200, max_file_size=1 << 19, n_files=6)
    wf, reset = _walk(files, names)
    want, wst = orc.replay(wf, reset)
    assert wst["status"] == 0
    bounds = [0, *cuts, len(wf)]
    shards = [(wf[a:b], reset[a:b]) for a, b in zip(bounds, bounds[1:])]
    shard_of_file = [s for s, (a, b) in enumerate(zip(bounds, bounds[1:])) for _ in range(a, b)]
    packed = _pack_shards(g, torch, shards, nparts)
    try:
        owners = [_merge_owner(torch, packed, p, packed[p % len(packed)][0]) for p in range(nparts)]
    finally:
        for c, *_ in packed:
            c.close()
    _check_merged(wf, owners, _global_keydir(wf, want), nparts, shard_of_file)


def test_merge_with_empty_shard(g, orc):
    import torch

    files, names = orc.gen_corpus(seed=72, val_fixed=0, key_min=8, key_max=16, key_universe=300,
                                  tomb_permille=100, max_file_size=1 << 18, n_files=3)
    wf, reset = _walk(files, names)
    want, _ = orc.replay(wf, reset)
    empty = np.zeros(0, dtype=np.uint8)
    # shard 1 holds one empty data file between the others
    shards = [(wf[:2], reset[:2]), ([empty], [True]), (wf[2:], reset[2:])]
    packed = _pack_shards(g, torch, shards, 2)
    try:
        assert sum(packed[1][3]) == 0
        owners = [_merge_owner(torch, packed, p, packed[0][0]) for p in range(2)]
    finally:
        for c, *_ in packed:
            c.close()
    files_all = wf[:2] + [empty] + wf[2:]
    recs = want.copy()
    recs["file"] = np.where(recs["file"] >= 2, recs["file"] + 1, recs["file"])
    _check_merged(files_all, owners, _global_keydir(files_all, recs), 2, [0, 0, 1, 2])


def test_merge_single_shard_is_live_keydir(g, orc):
    import torch

    files, names = orc.gen_corpus(seed=73, val_fixed=0, key_min=8, key_max=24, key_universe=5000,
                                  tomb_permille=50, max_file_size=1 << 20, n_files=4)
    wf, reset = _walk(files, names)
    packed = _pack_shards(g, torch, [(wf, reset)], 1)
    ctx = packed[0][0]
    try:
        live, _ = ctx.keydir()
        ents, _ = _merge_owner(torch, packed, 0, ctx)
    finally:
        ctx.close()
    assert len(ents) == len(live)
    for f in FIELDS:
        assert np.array_equal(ents["rec"][f], live[f]), f


def test_merge_rejects_foreign_entries(g, orc):
    import torch

    files, names = orc.gen_corpus(seed=74, val_fixed=100, key_min=8, key_max=8, key_universe=100,
                                  max_file_size=1 << 16, n_files=1)
    packed = _pack_shards(g, torch, [([files[0]], [False])], 1)
    ctx, ents, keys, counts, kb, _ = packed[0]
    try:
        e = ents[:counts[0] * 64].view(torch.int64).view(-1, 8)
        e[0, 1] += 3  # key_off no longer 8-aligned
        torch.cuda.synchronize()
        with pytest.raises(Exception):
            ctx.kd_merge(ents.data_ptr(), keys.data_ptr(), counts, kb)
        e[0, 1] -= 3
        e[1, 1] = kb[0]  # key past the blob
        torch.cuda.synchronize()
        with pytest.raises(Exception):
            ctx.kd_merge(ents.data_ptr(), keys.data_ptr(), counts, kb)
    finally:
        ctx.close()


def test_merge_keydir_rccl_world1(g, orc):
    """gocask_amd.shard.merge_keydir through a one-rank "nccl" (RCCL) group."""
    import os
    import socket

    import torch
    import torch.distributed as dist

    from gocask_amd import shard

    files, names = orc.gen_corpus(seed=75, val_fixed=0, key_min=8, key_max=24, key_universe=3000,
                                  tomb_permille=50, max_file_size=1 << 20, n_files=3)
    wf, reset = _walk(files, names)
    want, _ = orc.replay(wf, reset)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1)
    try:
        with g.ReplayContext() as ctx:
            ctx.load(wf, reset)
            ctx.run()
            base = shard.file_base(dist, len(wf), device="cuda")
            n, t = shard.merge_keydir(ctx, dist, base)
            ents, keys = ctx.kd_fetch_merged()
    finally:
        dist.destroy_process_group()
    assert base == 0 and n == len(ents)
    _check_merged(wf, [(ents, keys)], _global_keydir(wf, want), 1, [0] * len(wf))


def _rank_worker(rank, world, port, q):
    """One rank of a world-2 merge: its shard of the corpus on cuda:0, the
    exchange over gloo (staged through host memory)."""
    import os

    import torch
    import torch.distributed as dist

    import oracle as orc
    import gocask_amd as g
    from gocask_amd import shard

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        files, names = orc.gen_corpus(**MERGE_CORPUS)
        wf, reset = _walk(files, names)
        a, b = SPLIT[rank], SPLIT[rank + 1]
        with g.ReplayContext() as ctx:
            ctx.load(wf[a:b], reset[a:b])
            ctx.run()
            base = shard.file_base(dist, b - a)
            n, _ = shard.merge_keydir(ctx, dist, base)
            ents, keys = ctx.kd_fetch_merged()
        q.put((rank, base, n, ents.tobytes(), keys.tobytes()))
    except Exception as e:  # reported to the parent
        q.put((rank, None, repr(e), b"", b""))
    finally:
        dist.destroy_process_group()


MERGE_CORPUS = dict(seed=76, val_fixed=0, key_min=8, key_max=24, key_universe=2000, tomb_permille=150,
                    max_file_size=1 << 19, n_files=5)
SPLIT = [0, 2, 5]  # rank 0: files 0-1, rank 1: files 2-4 (walk order)


def test_merge_keydir_two_ranks(g, orc):
    """gocask_amd.shard.merge_keydir as bench.py runs it at N>1, with two
    processes (ranks) on one GPU and a gloo group: the owners' entries
    together must be the global keydir of all files in walk order."""
    import socket

    import torch.multiprocessing as mp

    from gocask_amd._lib import KD_ENTRY_DTYPE

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    for r, base, n, _, _ in res:
        assert base is not None, n
    assert [r[1] for r in res] == [0, 2]  # file_base: the files of lower ranks
    owners = [(np.frombuffer(e, dtype=KD_ENTRY_DTYPE), np.frombuffer(k, dtype=np.uint8)) for _, _, _, e, k in res]
    assert [len(o[0]) for o in owners] == [r[2] for r in res]
    files, names = orc.gen_corpus(**MERGE_CORPUS)
    wf, reset = _walk(files, names)
    want, _ = orc.replay(wf, reset)
    _check_merged(wf, owners, _global_keydir(wf, want), 2, [0, 0, 1, 1, 1])
    for p in procs:
        assert p.exitcode == 0


# ---------------------- exact sharding: planned cuts, startup error propagation ---
def _sharded_owners(g, torch, wf, reset, world, nparts):
    """plan_shards + one context per shard + resolve_status; only the shards
    up to the first startup error are packed (later ones send nothing)."""
    from gocask_amd import shard

    ranges = shard.plan_shards([len(f) for f in wf], reset, world)
    per = []
    for a, b in ranges:
        with g.ReplayContext() as ctx:
            if b > a:
                ctx.load(wf[a:b], reset[a:b])
                ctx.run()
                per.append(ctx.stats())
            else:
                per.append(dict(status=0, err_file=0, err_off=0, files_walked=0, final_last_offset=0, n_files=0))
    glob, contrib = shard.resolve_status(per)
    shards = [(wf[a:b], reset[a:b]) for (a, b), c in zip(ranges, contrib) if c]
    packed = _pack_shards(g, torch, shards, nparts)
    try:
        owners = [_merge_owner(torch, packed, p, packed[p % len(packed)][0]) for p in range(nparts)]
    finally:
        for c, *_ in packed:
            c.close()
    shard_of_file = [s for s, (a, b) in enumerate(ranges) for _ in range(a, b)]
    return glob, owners, shard_of_file


@pytest.mark.parametrize("world,nparts", [(2, 2), (3, 1), (4, 3)])
def test_sharded_startup_error_propagates(g, orc, world, nparts):
    import torch

    from golden_cases import load_case

    files, names = orc.gen_corpus(seed=77, val_fixed=0, key_min=8, key_max=16, key_universe=400,
                                  tomb_permille=150, max_file_size=1 << 17, n_files=5)
    wf, _ = _walk(files, names)
    _, bad, _ = load_case("partial_write_desync")  # "unexpected EOF" on a key read at offset 74
    wf = wf[:2] + [bad[0]] + wf[2:]
    reset = [True] * (len(wf) - 1) + [False]
    want, wst = orc.replay(wf, reset)
    assert wst["status"] == 1 and wst["err_file"] == 2
    glob, owners, shard_of_file = _sharded_owners(g, torch, wf, reset, world, nparts)
    assert (glob["status"], glob["err_file"], glob["err_off"], glob["files_walked"]) == (
        wst["status"], wst["err_file"], wst["err_off"], wst["files_walked"])
    _check_merged(wf, owners, _global_keydir(wf, want), nparts, shard_of_file)


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_keys_in_order_never_cuts_after_the_active_file(g, orc, world):
    # core/db_test.go:428-471: the active "data" is walked first and does not
    # reset lastOffset, so foobar in data01 has ValuePos 66; a cut right after
    # "data" would give 22
    import torch

    from golden_cases import load_case

    from gocask_amd import shard

    meta, files, reset = load_case("keys_in_order")
    assert reset[0] is False
    ranges = shard.plan_shards([len(f) for f in files], reset, world)
    assert all(a != 1 for a, _ in ranges)
    want, wst = orc.replay(files, reset)
    glob, owners, shard_of_file = _sharded_owners(g, torch, files, reset, world, 2)
    assert glob["status"] == 0 and glob["final_last_offset"] == wst["final_last_offset"] == meta["final_last_offset"]
    kd = _global_keydir(files, want)
    _check_merged(files, owners, kd, 2, shard_of_file)
    assert int(kd[b"foobar"]["value_pos"]) == 66


@pytest.mark.parametrize("key_seed", [0, 4])
def test_encode_files_matches_oracle_one_file_corpora(g, orc, key_seed):
    # BASELINE C4's generator: file n is a one-file corpus with seed + n; with
    # key_seed its keys come from one universe shared by all files
    kw = dict(seed=4, val_fixed=0, key_min=8, key_max=24, key_universe=2000, tomb_permille=10, flip_permille=10,
              max_file_size=1 << 20, n_files=1, key_seed=key_seed)
    ids = [3, 0, 11]
    with g.ReplayContext() as ctx:
        info = ctx.encode_files(ids, last_is_active=True, **kw)
        files = []
        for k, n in enumerate(ids):
            want_f, want_names = orc.gen_corpus(**{**kw, "seed": 4 + n, "key_file": n})
            assert len(want_f) == 1 and int(info["sizes"][k]) == len(want_f[0])
            got = ctx.read_file(k, 0, len(want_f[0]))
            assert np.array_equal(got, want_f[0]), n
            files.append(want_f[0])
        ctx.run()
        recs, st = ctx.fetch()
    want, wst = orc.replay(files, [True, True, False])
    assert st["status"] == 0 and len(recs) == len(want) == info["n_ops"]
    for f in FIELDS:
        assert np.array_equal(recs[f], want[f]), f
    assert st["final_last_offset"] == wst["final_last_offset"] == len(files[-1])


def _c4_files(orc, world, files_per_rank, universe, max_file_size, tomb_permille=10):
    """The C4 corpus spec (bench.py CONFIGS["c4"]: per-file seed 4 + n, keys
    from one universe with key_seed 4) at a small file size: (files in walk
    order, reset flags, shard ranges) for `world` ranks."""
    from gocask_amd import shard

    kw = dict(seed=4, key_seed=4, val_fixed=0, key_min=8, key_max=24, key_universe=universe,
              tomb_permille=tomb_permille, max_file_size=max_file_size, n_files=1)
    wf, ranges = [], []
    for r in range(world):
        ids, _ = shard.c4_file_ids(world, r, files_per_rank)
        ranges.append((len(wf), len(wf) + len(ids)))
        for n in ids:
            f, _ = orc.gen_corpus(**{**kw, "seed": 4 + n, "key_file": n})
            wf.append(f[0])
    reset = [i + 1 < len(wf) for i in range(len(wf))]
    return wf, reset, ranges


@pytest.mark.parametrize("tomb_permille", [10, 150])
def test_merge_c4_keys_shared_across_shards(g, orc, tomb_permille):
    """C4 key density (a universe of half the records, shared by every file):
    later shards overwrite and delete keys of earlier ones, and the merged
    keydir equals keyDir.set / unset over all files in walk order
    (core/keydir.go:22-49)."""
    import torch

    wf, reset, ranges = _c4_files(orc, 4, 2, universe=1200, max_file_size=1 << 20, tomb_permille=tomb_permille)
    want, wst = orc.replay(wf, reset)
    assert wst["status"] == 0
    assert 1500 < len(want) < 4000  # the universe is about half the records
    shard_of_file = [s for s, (a, b) in enumerate(ranges) for _ in range(a, b)]
    # keys cross shards: some key's last word (a Put or a Delete) comes from a
    # later shard than one of its earlier Puts
    first_put, crosses, deletes_across = {}, 0, 0
    for r in want:
        o = int(r["rec_off"]) + 16
        key = bytes(wf[int(r["file"])][o:o + int(r["key_len"])])
        s = shard_of_file[int(r["file"])]
        if key in first_put and first_put[key] < s:
            crosses += 1
            deletes_across += int(r["flags"]) & 1
        if not int(r["flags"]) & 1:
            first_put.setdefault(key, s)
    assert crosses > 100 and deletes_across > 0, (crosses, deletes_across)
    shards = [(wf[a:b], reset[a:b]) for a, b in ranges]
    packed = _pack_shards(g, torch, shards, 4)
    try:
        owners = [_merge_owner(torch, packed, p, packed[p][0]) for p in range(4)]
    finally:
        for c, *_ in packed:
            c.close()
    _check_merged(wf, owners, _global_keydir(wf, want), 4, shard_of_file)
