"""Keydir merge across GPUs: the one exchange step of the
sharded replay.

Files shard over ranks in walk order (rank r holds a contiguous run of files,
every file but the last rank's last one resets lastOffset), so every rank
replays its shard with no collective.  The keydir the reference builds over
all files (keyDir.set / unset in walk order, core/keydir.go:22-49) is then:

  1. per rank, the shard's keydir with tombstones kept (gck_ctx_keydir with
     GCK_KD_KEEP_TOMBSTONES): a shard's last word on a key may be a delete that
     hides an earlier shard's Put;
  2. entries partitioned by key hash over the ranks (gck_kd_pack);
  3. one all-to-all of the entries and one of their key bytes (RCCL over xGMI
     with the "nccl" backend; gloo on CPU for the host-logic tests);
  4. per owner, the highest shard's entry of each key wins, a winning
     tombstone drops the key (gck_kd_merge).

The owners' merged entries together are the global keydir; each key lives on
exactly one owner.

Exactness across the cuts (core/db.go:110-138):
  - plan_shards only cuts after a file that resets lastOffset
    (Name() != activeFile.Name(), core/db.go:117-119), so no shard needs a
    lastOffset carried in from another;
  - the first startup error aborts the whole walk (core/db.go:134-138,
    internal/fs/disk.go:134-141): resolve_status finds the lowest shard that
    failed; its records before the error count, later shards contribute
    nothing, and the global status is that error.
"""
from __future__ import annotations

import time

KD_ENTRY_BYTES = 64
GCK_EUNEXPECTED_EOF = 1


def plan_shards(sizes, reset_after, world):
    """Cut files in walk order into `world` contiguous ranges [(a, b), ...]
    (file b excluded) of about equal bytes.  A cut at i (between files i-1
    and i) is allowed only if file i-1 resets lastOffset (reset_after), so
    each shard replays exactly as the global walk would; ranges may be empty
    (more ranks than allowed cuts)."""
    n = len(sizes)
    if world < 1:
        raise ValueError("world must be >= 1")
    prefix = [0]
    for x in sizes:
        prefix.append(prefix[-1] + int(x))
    ok = [i for i in range(1, n) if reset_after[i - 1]]  # allowed cut positions
    cuts, lo = [], 0
    for k in range(1, world):
        target = prefix[n] * k / world
        cand = [i for i in ok if i >= lo]
        if not cand:
            cuts.append(n)
            continue
        best = min(cand, key=lambda i: (abs(prefix[i] - target), i))
        cuts.append(best)
        lo = best
    bounds = [0] + cuts + [n]
    return [(bounds[r], max(bounds[r], bounds[r + 1])) for r in range(world)]


def resolve_status(per_rank):
    """Global outcome of a sharded replay from each rank's run outcome, in
    rank (= walk) order: dicts with status, err_file, err_off, files_walked,
    final_last_offset, n_files.  Returns (global dict, contributes[rank])."""
    base, out, contrib = 0, None, []
    last = 0
    for st in per_rank:
        if out is not None:  # after the first startup error: nothing counts
            contrib.append(False)
            continue
        contrib.append(True)
        if st["status"] == GCK_EUNEXPECTED_EOF:
            out = dict(status=GCK_EUNEXPECTED_EOF, err_file=base + st["err_file"], err_off=st["err_off"],
                       files_walked=base + st["files_walked"], final_last_offset=st["final_last_offset"])
        elif st["n_files"]:
            last = st["final_last_offset"]  # cuts follow resetting files: the last shard's value
        base += st["n_files"]
    if out is None:
        out = dict(status=0, err_file=0, err_off=0, files_walked=base, final_last_offset=last)
    return out, contrib


def c4_file_ids(world, rank, files_per_rank=16, ts_base=1700000000):
    """BASELINE C4 shards: one corpus of files_per_rank * world files named
    data_<n>_<ts_base+n>, walked in bytewise name order, cut into
    contiguous ranges; rank's creation ids in walk order, and whether its
    last file is the active one (the globally last entry)."""
    total = files_per_rank * world
    names = sorted((f"data_{n}_{ts_base + n}.csk", n) for n in range(total))
    reset = [i + 1 < total for i in range(total)]
    a, b = plan_shards([1] * total, reset, world)[rank]
    return [n for _, n in names[a:b]], b == total and b > a


def exchange(dist, send, send_splits, group=None):
    """All-to-all of a flat uint8 tensor laid out as consecutive per-rank parts
    of send_splits bytes.  Returns (received tensor, received split sizes), the
    parts in rank order, on send's device.  RCCL moves device tensors
    directly; a gloo group (CPU tests, ranks sharing one GPU) is staged
    through host memory."""
    import torch

    if send.is_cuda and dist.get_backend(group) == "gloo":
        recv, rs = exchange(dist, send.cpu(), send_splits, group)
        return recv.to(send.device), rs
    ss = torch.tensor([int(x) for x in send_splits], dtype=torch.int64, device=send.device)
    rs = torch.empty_like(ss)
    dist.all_to_all_single(rs, ss, group=group)
    recv_splits = [int(x) for x in rs.tolist()]
    recv = torch.empty(max(sum(recv_splits), 1), dtype=torch.uint8, device=send.device)
    if send.numel() < max(sum(send_splits), 1):
        raise ValueError("send buffer shorter than its splits")
    dist.all_to_all_single(recv[:sum(recv_splits)], send[:sum(send_splits)],
                           output_split_sizes=recv_splits, input_split_sizes=[int(x) for x in send_splits],
                           group=group)
    return recv, recv_splits


def file_base(dist, n_files, group=None, device="cpu"):
    """Global walk index of this rank's first file: the files of lower ranks."""
    import torch

    world = dist.get_world_size(group)
    if dist.get_backend(group) == "gloo":
        device = "cpu"
    t = torch.tensor([int(n_files)], dtype=torch.int64, device=device)
    all_n = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(all_n, t, group=group)
    return sum(int(x.item()) for x in all_n[:dist.get_rank(group)])


def gather_status(ctx, dist, group=None):
    """Every rank's run outcome (ctx.stats()) -> resolve_status over ranks."""
    import torch

    st = ctx.stats()
    dev = "cpu" if dist.get_backend(group) == "gloo" else torch.device("cuda", torch.cuda.current_device())
    keys = ("status", "err_file", "err_off", "files_walked", "final_last_offset", "n_files")
    t = torch.tensor([int(st[k]) for k in keys], dtype=torch.int64, device=dev)
    world = dist.get_world_size(group)
    parts = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(parts, t, group=group)
    return resolve_status([dict(zip(keys, (int(x) for x in p.tolist()))) for p in parts])


def merge_keydir(ctx, dist, base, group=None):
    """Global keydir entries owned by this rank, merged on its GPU after
    ctx.run(): returns (n_live, dict of phase seconds and the global run
    outcome).  The entries stay on the device; ctx.kd_fetch_merged() copies
    them (KD_ENTRY_DTYPE) and their keys.  base: the global walk index of this
    rank's first file (file_base()).  Ranks after the first startup error
    send nothing (resolve_status)."""
    import torch

    rank, world = dist.get_rank(group), dist.get_world_size(group)
    dev = torch.device("cuda", torch.cuda.current_device())
    t0 = time.perf_counter()
    glob, contrib = gather_status(ctx, dist, group)
    if contrib[rank]:
        ctx.keydir(keep_tombstones=True, fetch=False)
        counts, kbytes = ctx.kd_pack_sizes(world)
    else:
        counts, kbytes = [0] * world, [0] * world
    ne, nk = sum(counts), sum(kbytes)
    ents = torch.empty(max(ne * KD_ENTRY_BYTES, 1), dtype=torch.uint8, device=dev)
    keys = torch.empty(max(nk, 1), dtype=torch.uint8, device=dev)
    torch.cuda.current_stream().synchronize()  # the allocations, before the library's stream writes them
    if ne or nk:
        ctx.kd_pack(rank, base, ents.data_ptr(), ne, keys.data_ptr(), nk)
    t1 = time.perf_counter()
    r_ents, r_esplit = exchange(dist, ents, [c * KD_ENTRY_BYTES for c in counts], group)
    r_keys, r_ksplit = exchange(dist, keys, kbytes, group)
    torch.cuda.current_stream().synchronize()
    t2 = time.perf_counter()
    n_live, _ = ctx.kd_merge(r_ents.data_ptr(), r_keys.data_ptr(), [b // KD_ENTRY_BYTES for b in r_esplit],
                             r_ksplit)
    t3 = time.perf_counter()
    return n_live, dict(local=t1 - t0, exchange=t2 - t1, merge=t3 - t2,
                        sent_bytes=ne * KD_ENTRY_BYTES + nk, status=glob)
