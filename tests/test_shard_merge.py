"""Host logic of the keydir merge across shards on CPU.

- gocask_amd.shard.exchange / file_base over a world-size-2 gloo group: the
  all-to-all that carries packed keydir partitions between ranks;
- the merge rule itself on the oracle's records: per-shard keydirs with
  tombstones kept, partitioned by key, highest shard wins, winning deletes
  dropped == keyDir.set / unset over every file in walk order
  (core/keydir.go:22-49).  The GPU kernels doing this are checked against the
  same expectation in test_gpu_merge.py.
"""
import os
import socket
import sys
import zlib

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _exchange_worker(rank, world, port, out):
    import torch
    import torch.distributed as dist

    from gocask_amd import shard

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # rank r sends (r+1)*(d+1) bytes of value 16*r+d to rank d; rank 1's
        # part for rank 0 is empty
        splits = [0 if (rank == 1 and d == 0) else (rank + 1) * (d + 1) for d in range(world)]
        send = torch.cat([torch.full((n,), 16 * rank + d, dtype=torch.uint8) for d, n in enumerate(splits)])
        recv, rsplits = shard.exchange(dist, send, splits)
        base = shard.file_base(dist, 3 + rank)
        out.put((rank, bytes(recv[:sum(rsplits)].tolist()), rsplits, base))
    finally:
        dist.destroy_process_group()


def test_exchange_two_ranks_gloo():
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_exchange_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, b0, s0, base0), (r1, b1, s1, base1) = res
    assert s0 == [1, 0] and b0 == bytes([0])  # from rank 0: 1 byte; from rank 1: nothing
    assert s1 == [2, 4] and b1 == bytes([1, 1]) + bytes([17] * 4)
    assert (base0, base1) == (0, 3)


def _keydir_with_tombstones(files, recs, file_base):
    """A shard's keydir, deletes kept as markers: {key: (global file, rec)}."""
    kd = {}
    for r in recs:
        o = int(r["rec_off"]) + 16
        key = bytes(files[int(r["file"])][o:o + int(r["key_len"])])
        kd[key] = (int(r["file"]) + file_base, r)
    return kd


@pytest.mark.parametrize("cuts,nparts", [((2,), 2), ((1, 2, 4), 3), ((3,), 5)])
def test_sharded_merge_rule_equals_global_keydir(orc, cuts, nparts):
    files, names = orc.gen_corpus(seed=81, val_fixed=0, key_min=8, key_max=16, key_universe=400,
                                  tomb_permille=200, max_file_size=1 << 16, n_files=5)
    walk = sorted(range(len(files)), key=lambda i: names[i])
    wf = [files[i] for i in walk]
    reset = [i + 1 < len(wf) for i in range(len(wf))]
    want, _ = orc.replay(wf, reset)
    glob = {}
    for r in want:
        o = int(r["rec_off"]) + 16
        key = bytes(wf[int(r["file"])][o:o + int(r["key_len"])])
        if int(r["flags"]) & 1:
            glob.pop(key, None)
        else:
            glob[key] = (int(r["file"]), int(r["rec_off"]))

    bounds = [0, *cuts, len(wf)]
    owners = [[] for _ in range(nparts)]  # what each owner receives, in shard order
    for s, (a, b) in enumerate(zip(bounds, bounds[1:])):
        recs, st = orc.replay(wf[a:b], reset[a:b])
        assert st["status"] == 0
        # every shard but the last ends on a resetting file: its value_pos
        # equal the global replay's
        for key, (f, r) in _keydir_with_tombstones(wf[a:b], recs, a).items():
            owners[zlib.crc32(key) % nparts].append((s, key, f, r))
    merged = {}
    for p, got in enumerate(owners):
        win = {}
        for s, key, f, r in got:  # shard order: a later shard replaces
            win[key] = (f, r)
        for key, (f, r) in win.items():
            assert key not in merged
            if not int(r["flags"]) & 1:
                merged[key] = (f, int(r["rec_off"]))
    assert merged == glob


# ------------------------------------------------ shard planning (exact cuts) ---
def test_plan_shards_cuts_only_after_resetting_files():
    import random

    from gocask_amd import shard

    rng = random.Random(5)
    for _ in range(300):
        n = rng.randint(0, 12)
        sizes = [rng.randint(0, 100) for _ in range(n)]
        reset = [rng.random() < 0.7 for _ in range(n)]
        world = rng.randint(1, 6)
        ranges = shard.plan_shards(sizes, reset, world)
        assert len(ranges) == world and ranges[0][0] == 0 and ranges[-1][1] == n
        for (a, b), (c, _) in zip(ranges, ranges[1:]):
            assert a <= b == c  # contiguous, in walk order
        for a, b in ranges[1:]:
            assert a == n or a == 0 or reset[a - 1], (sizes, reset, ranges)


def test_plan_shards_balances_bytes():
    from gocask_amd import shard

    assert shard.plan_shards([10] * 16, [True] * 15 + [False], 4) == [(0, 4), (4, 8), (8, 12), (12, 16)]
    # the active file walked first (core/db_test.go:428-471): no cut right after it
    assert shard.plan_shards([41, 25, 25], [False, True, True], 3) == [(0, 2), (2, 2), (2, 3)]
    assert shard.plan_shards([5, 5], [True, False], 1) == [(0, 2)]


def _status(st, n_files):
    return dict(status=st["status"], err_file=st["err_file"], err_off=st["err_off"],
                files_walked=st["files_walked"], final_last_offset=st["final_last_offset"], n_files=n_files)


@pytest.mark.parametrize("world", [2, 3, 5])
def test_sharded_replay_with_startup_error_equals_global(orc, world):
    """A startup error in one shard aborts the walk for every later shard
    (core/db.go:134-138, disk.go:134-141): resolve_status + the merge rule on
    the oracle's per-shard records == the oracle's global replay."""
    from golden_cases import load_case

    from gocask_amd import shard

    files, names = orc.gen_corpus(seed=83, val_fixed=0, key_min=8, key_max=16, key_universe=300,
                                  tomb_permille=150, max_file_size=1 << 15, n_files=6)
    wf = [files[i] for i in sorted(range(len(files)), key=lambda i: names[i])]
    _, bad, _ = load_case("partial_write_desync")
    wf = wf[:3] + [bad[0]] + wf[3:]
    reset = [True] * (len(wf) - 1) + [False]
    want, wst = orc.replay(wf, reset)
    assert wst["status"] == 1 and wst["err_file"] == 3
    ranges = shard.plan_shards([len(f) for f in wf], reset, world)
    per, recs_of = [], []
    for a, b in ranges:
        recs, st = orc.replay(wf[a:b], reset[a:b]) if b > a else (want[:0], dict(
            status=0, err_file=0, err_off=0, files_walked=0, final_last_offset=0))
        per.append(_status(st, b - a))
        recs_of.append((a, recs))
    glob, contrib = shard.resolve_status(per)
    assert glob["status"] == wst["status"] and glob["err_file"] == wst["err_file"]
    assert glob["err_off"] == wst["err_off"] and glob["files_walked"] == wst["files_walked"]
    merged = {}
    for (a, recs), c in zip(recs_of, contrib):
        if not c:
            continue
        for key, (f, r) in _keydir_with_tombstones(wf[a:], recs, a).items():
            if int(r["flags"]) & 1:
                merged.pop(key, None)
            else:
                merged[key] = (f, int(r["rec_off"]), int(r["value_pos"]))
    glob_kd = {}
    for r in want:
        o = int(r["rec_off"]) + 16
        key = bytes(wf[int(r["file"])][o:o + int(r["key_len"])])
        if int(r["flags"]) & 1:
            glob_kd.pop(key, None)
        else:
            glob_kd[key] = (int(r["file"]), int(r["rec_off"]), int(r["value_pos"]))
    assert merged == glob_kd


def test_resolve_status_without_errors():
    from gocask_amd import shard

    ok = lambda n, last: dict(status=0, err_file=0, err_off=0, files_walked=n, final_last_offset=last, n_files=n)
    g, c = shard.resolve_status([ok(2, 0), ok(0, 0), ok(3, 77), ok(0, 0)])
    assert g == dict(status=0, err_file=0, err_off=0, files_walked=5, final_last_offset=77) and all(c)


def test_c4_shards_cover_the_corpus_in_walk_order():
    from gocask_amd import shard

    for world in (1, 2, 4, 8):
        total = 16 * world
        names = sorted(f"data_{n}_{1700000000 + n}.csk" for n in range(total))
        got, actives = [], []
        for r in range(world):
            ids, last_active = shard.c4_file_ids(world, r)
            assert len(ids) == 16
            got += ids
            actives.append(last_active)
        assert [f"data_{n}_{1700000000 + n}.csk" for n in got] == names
        assert actives == [False] * (world - 1) + [True]


class _FakeCtx:
    def __init__(self, st):
        self._st = st

    def stats(self):
        return self._st


def _status_worker(rank, world, port, out):
    import torch.distributed as dist

    from gocask_amd import shard

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        st = [dict(status=0, err_file=0, err_off=0, files_walked=2, final_last_offset=0, n_files=2),
              dict(status=1, err_file=1, err_off=74, files_walked=2, final_last_offset=9, n_files=3)][rank]
        out.put((rank,) + shard.gather_status(_FakeCtx(st), dist))
    finally:
        dist.destroy_process_group()


def test_gather_status_two_ranks_gloo():
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_status_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for _, g, c in res:
        assert g == dict(status=1, err_file=3, err_off=74, files_walked=4, final_last_offset=9) and c == [True, True]


def test_library_plan_shards_equals_python():
    """gck_plan_shards (the C-ABI planner gck_replay_multi uses; host only, no
    device) cuts exactly as gocask_amd.shard.plan_shards."""
    import random

    import gocask_amd as g
    from gocask_amd import shard

    rng = random.Random(5)
    for _ in range(2000):
        n, w = rng.randint(0, 24), rng.randint(1, 9)
        sizes = [rng.choice([0, 1, 4096, rng.randint(0, 1 << 31)]) for _ in range(n)]
        reset = [rng.random() < 0.85 for _ in range(n)]
        assert g.plan_shards(sizes, reset, w) == shard.plan_shards(sizes, reset, w), (sizes, reset, w)
