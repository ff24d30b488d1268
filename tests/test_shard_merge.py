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
