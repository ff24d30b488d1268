"""Multi-rank bench logic on CPU (gloo, world size 2): each rank gets its own
shard of independent files and the job time is the slowest rank's, the bytes
the sum of all ranks' (bench.py; SURVEY.md §8e: files shard with no data-path
collective)."""
import os
import socket
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out):
    import torch.distributed as dist

    import bench

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cfg = bench.shard_config("c3", rank)
        # rank r pretends to take 1+r seconds over 100*(r+1) bytes
        t, b = bench.reduce_over_ranks(dist, 1.0 + rank, 100 * (rank + 1), "cpu")
        out.put((rank, cfg["seed"], t, b))
    finally:
        dist.destroy_process_group()


def test_two_rank_shards_and_reduction():
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, s0, t0, b0), (r1, s1, t1, b1) = res
    assert s0 != s1  # distinct shards
    assert t0 == t1 == 2.0  # max over ranks
    assert b0 == b1 == 300.0  # sum over ranks


def test_shards_are_disjoint_corpora(orc):
    """Shard seeds give different files (same spec): a small C3-shaped config."""
    import bench

    kw0, kw1 = bench.shard_config("c3", 0), bench.shard_config("c3", 1)
    small = dict(max_file_size=1 << 20, n_files=1, key_universe=1000)
    f0, _ = orc.gen_corpus(**{**kw0, **small})
    f1, _ = orc.gen_corpus(**{**kw1, **small})
    assert bytes(f0[0][:4096]) != bytes(f1[0][:4096])


def test_cpu_baseline_variants(orc):
    """bench.py's cpu_baseline: SURVEY.md §8d's three variants on a tiny sample."""
    import bench

    out = bench.cpu_baseline("c3", 4 << 20, max_threads=2, min_s=0.05, mt_file_bytes=2 << 20)
    assert out["kind"] == "port" and out["cores"] == 1 and out["value"] > 0
    v = out["variants"]
    assert set(v) == {"ref_faithful", "ref_crc", "all_cores"}
    assert v["ref_faithful"]["value"] == out["value"] and v["all_cores"]["cores"] == 2  # the reference replay: no CRC
    assert all(x["value"] > 0 for x in v.values())
