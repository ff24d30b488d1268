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
"""
from __future__ import annotations

import time

KD_ENTRY_BYTES = 64


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


def merge_keydir(ctx, dist, base, group=None):
    """Global keydir entries owned by this rank, merged on its GPU after
    ctx.run(): returns (n_live, dict of phase seconds).  The entries stay on the
    device; ctx.kd_fetch_merged() copies them (KD_ENTRY_DTYPE) and their keys.
    base: the global walk index of this rank's first file (file_base())."""
    import torch

    rank, world = dist.get_rank(group), dist.get_world_size(group)
    dev = torch.device("cuda", torch.cuda.current_device())
    t0 = time.perf_counter()
    ctx.keydir(keep_tombstones=True, fetch=False)
    counts, kbytes = ctx.kd_pack_sizes(world)
    ne, nk = sum(counts), sum(kbytes)
    ents = torch.empty(max(ne * KD_ENTRY_BYTES, 1), dtype=torch.uint8, device=dev)
    keys = torch.empty(max(nk, 1), dtype=torch.uint8, device=dev)
    torch.cuda.current_stream().synchronize()  # the allocations, before the library's stream writes them
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
                        sent_bytes=ne * KD_ENTRY_BYTES + nk)
