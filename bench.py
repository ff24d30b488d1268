#!/usr/bin/env python3
"""Benchmark: device-resident cold-start replay throughput (BASELINE.json metric).

A "step" is one full replay of the resident corpus: speculative boundary scan,
chain walk, validation, record table, CRC of every value, verdict + tuples
(gck_ctx_run).  The corpus is synthetic (DESIGN.md "Corpus"), encoded straight
into HBM by the device encoder before timing starts.

  python bench.py [--gpus N --steps K --warmup W --config c3]
  N>1: python bench.py --gpus N starts the N rank processes itself (a
       torch.distributed.run child, launched before this process touches a
       GPU; rank 0's JSON line passes through), or under a launcher:
       python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

N = 1 times C3 (BASELINE's metric config).  N > 1 times C4: one corpus of
16 x N files of 2 GiB (per-file seed 4 + n), cut into N contiguous walk-order
shards, one per rank (weak scaling; no data-path collective: the files are
independent).
After the timed replays, N>1 runs also time the keydir merge across ranks (the
path's one exchange step, RCCL all-to-all; reported as "keydir_merge", not
part of value).  Rank 0 prints one JSON line.

  python bench.py --gpus N --lib-multi   the drop-in multi-GPU path instead:
       ONE process, a ReplayContext per device holding rank r's C4 shard,
       the replays from one host thread each, then the library's own keydir
       exchange + merge (gck_ctx_multi_keydir: RCCL across devices, as
       gck_replay_multi), reported as "keydir_merge_lib".  More ranks than
       visible GPUs share them (a loopback rehearsal: device copies instead of
       RCCL).  The default N>1 run ends with this mode as a child process of
       rank 0 (after every rank has released its GPU) and reports its
       keydir_merge_lib beside the torch path's keydir_merge.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

GiB = 1 << 30
C4_KEYS_PER_FILE = 312_500  # C4's key universe = this x the corpus's files
CONFIGS = {
    # BASELINE.json configs[]: C1 CPU plumbing, C2 8 GiB fixed 4 KiB, C3 32 GiB Zipf, C5 = C3 + 1% flips
    "c1": dict(seed=1, val_fixed=1024, key_min=16, key_max=16, max_file_size=64 << 20, n_files=1),
    "c2": dict(seed=2, val_fixed=4096, key_min=16, key_max=16, max_file_size=8 << 30, n_files=1),
    "c3": dict(seed=3, val_fixed=0, key_min=8, key_max=24, key_universe=5_000_000, tomb_permille=10,
               max_file_size=2 << 30, n_files=16),
    "c5": dict(seed=3, val_fixed=0, key_min=8, key_max=24, key_universe=5_000_000, tomb_permille=10,
               flip_permille=10, max_file_size=2 << 30, n_files=16),
    # C4: one corpus of 16 x N files (8 GPUs: 128 x 2 GiB = 256 GiB), file n a
    # one-file C3-spec corpus (ops, values, deletes from seed 4 + n; SURVEY.md
    # §8d) whose keys come from ONE corpus-wide universe (key_seed 4, 50 % of
    # the records as C3: 312,500 ids per file), so keys repeat across files and
    # shards; cut into N contiguous walk-order shards (shard.c4_file_ids)
    "c4": dict(seed=4, key_seed=4, val_fixed=0, key_min=8, key_max=24, key_universe=C4_KEYS_PER_FILE,
               tomb_permille=10, max_file_size=2 << 30, n_files=1),
}
C4_FILES_PER_GPU = 16
DESCR = {
    "c1": "C1: 1 x 64 MiB file, 16 B keys, 1 KiB values",
    "c2": "C2: 1 x 8 GiB file, 16 B keys, 4 KiB values",
    "c3": "C3: 32 GiB = 16 x 2 GiB rotated files, 8-24 B keys, Zipf(1.1) 64 B-64 KiB values, 1% tombstones",
    "c5": "C5: C3 + 1% single-bit flips in values",
    "c4": "C4: {n} x 2 GiB files (C3 spec, per-file seed 4+n, one corpus-wide key universe), one corpus cut into {g} contiguous walk-order shards",
}
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def usable_cpus():
    """CPUs this process may use: its affinity mask, capped by a cgroup CPU
    quota (cpu.max) and by OMP_NUM_THREADS when set (the GPU box gives each
    job a share of a larger machine).  Returns (usable, dict of the sources)."""
    src = {"nproc": os.cpu_count() or 1}
    try:
        src["affinity"] = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        src["affinity"] = src["nproc"]
    n = src["affinity"]
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            src["cgroup_quota"] = max(1, int(int(quota) / int(period)))
            n = min(n, src["cgroup_quota"])
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        src["omp_num_threads"] = int(omp)
        n = min(n, int(omp))
    return max(1, n), src


def _timed(fn, min_s=4.0):
    reps, t = 0, 0.0
    while t < min_s or reps < 1:
        t0 = time.perf_counter()
        out = fn()
        t += time.perf_counter() - t0
        reps += 1
    return out, reps, t


def cpu_baseline(cfg_name, sample_bytes, max_threads=None, min_s=4.0, mt_file_bytes=256 << 20):
    """Oracle (C port of the reference replay) on host cores, on bounded samples
    of the same workload (SURVEY.md §8d's three variants):
      ref_faithful  1 thread: header decode, every byte through a 4 KiB buffer (bufio), key,
                    hash-map keydir, no CRC -- what the reference's replay does
                    (core/db.go:125-178 checks no CRC; Get does, lazily): the `value`;
      ref_crc       1 thread: the same plus the CRC verdict per record, by PCLMULQDQ
                    folding as Go's hash/crc32 does on amd64 (ieeeCLMUL; oracle
                    orc_crc32_clmul), for comparison with the GPU's verdict-on-every-record;
      all_cores     one thread per file on every usable CPU (usable_cpus()), + CRC,
                    a keydir per file (no cross-file merge).
    The oracle is a C port: Go's reflective binary.Read and per-record
    allocations (core/db.go:145-178) are not in it, so ref_faithful likely
    overstates the Go reference's speed (kind "port")."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    from concurrent.futures import ThreadPoolExecutor

    oracle.build()
    kw = dict(CONFIGS[cfg_name])
    kw["n_files"] = 1
    kw["max_file_size"] = min(kw["max_file_size"], sample_bytes)
    files, _ = oracle.gen_corpus(**kw)
    nbytes = sum(len(f) for f in files)
    (_, st), reps, t = _timed(lambda: oracle.baseline(files, [False]), min_s)
    (_, _), reps0, t0 = _timed(lambda: oracle.baseline(files, [False], verify_crc=False), min_s)
    what = f"first file of the {cfg_name.upper()} corpus ({nbytes / GiB:.2f} GiB, {st['n_recs']} records)"
    variants = dict(
        ref_faithful=dict(value=round(nbytes * reps0 / t0 / GiB, 3), cores=1,
                          sample=what + ", bytes through a 4 KiB buffer, no CRC (the reference's replay)"),
        ref_crc=dict(value=round(nbytes * reps / t / GiB, 3), cores=1,
                     sample=what + ", + CRC verdict per record (PCLMULQDQ folding, Go's amd64 hash/crc32 class)"),
    )
    nt, cpus = usable_cpus()
    nt = min(nt, max_threads) if max_threads else nt  # (tests: a small sample)
    nproc = cpus["nproc"]
    kw_mt = dict(CONFIGS[cfg_name])
    kw_mt["n_files"] = nt
    kw_mt["max_file_size"] = min(kw_mt["max_file_size"], mt_file_bytes)
    mfiles, _ = oracle.gen_corpus(**kw_mt)
    mbytes = sum(len(f) for f in mfiles)
    with ThreadPoolExecutor(max_workers=nt) as ex:
        def run_all():
            return list(ex.map(lambda f: oracle.baseline([f], [True]), mfiles))
        _, reps2, t2 = _timed(run_all, min_s)
    variants["all_cores"] = dict(value=round(mbytes * reps2 / t2 / GiB, 3), cores=nt,
                                 sample=f"{len(mfiles)} files of the {cfg_name.upper()} spec ({mbytes / GiB:.2f} GiB), "
                                        f"one thread per file, + CRC verdict (CLMUL), a keydir per file")
    return dict(value=variants["ref_faithful"]["value"], unit="GiB/s", cores=1, kind="port",
                sample=what + f", single-thread oracle replay as the reference does it (4 KiB buffered reads, "
                              f"header decode, key copy, hash-map keydir, no CRC), {reps0} pass(es)",
                variants=variants, nproc=nproc, usable_cpus=nt, cpu_sources=cpus, cpu_model=_cpu_model())


def host_inclusive(g, ctx, info, steps):
    """The path as the north star states it: files in (pinned, page-locked)
    host memory, tuples back in host memory.  Two ways:
      sequential  gck_ctx_load (H2D of every file), gck_ctx_run, gck_ctx_fetch_into;
      pipelined   gck_replay_into: all H2D copies queued at once, each group of
                  files (>= 1 GiB) replayed as soon as it is resident, the tuples
                  of all groups gathered into the caller's pinned array."""
    import numpy as np

    nf = info["n_files"]
    sizes = [int(info["sizes"][info["walk_order"][w]]) for w in range(nf)]
    host = np.empty(sum(sizes), dtype=np.uint8)
    g.host_register(host)
    views, off = [], 0
    for w, n in enumerate(sizes):
        views.append(ctx.read_file(w, 0, n, out=host[off:off + n]))
        off += n
    reset = [w + 1 < nf for w in range(nf)]
    recs = np.empty(ctx.stats()["n_recs"], dtype=g.REC_DTYPE)
    g.host_register(recs)
    t = dict(h2d=0.0, run=0.0, d2h=0.0)
    n_recs = 0
    for _ in range(steps):
        t0 = time.perf_counter()
        ctx.load(views, reset)
        t1 = time.perf_counter()
        ctx.run()
        t2 = time.perf_counter()
        n_recs = ctx.fetch_into(recs)
        t3 = time.perf_counter()
        t["h2d"] += t1 - t0
        t["run"] += t2 - t1
        t["d2h"] += t3 - t2
    total = sum(t.values())
    g.replay_into(views, recs, reset)  # warm-up (context creation, allocations)
    tp = 0.0
    for _ in range(steps):
        t0 = time.perf_counter()
        st = g.replay_into(views, recs, reset)
        tp += time.perf_counter() - t0
    assert st["n_recs"] == n_recs
    g.host_unregister(host)
    g.host_unregister(recs)
    return dict(value=round(host.nbytes * steps / tp / GiB, 3), unit="GiB/s", steps=steps,
                ms_per_step=round(tp / steps * 1e3, 2), tuple_bytes=n_recs * 40,
                sequential=dict(value=round(host.nbytes * steps / total / GiB, 3),
                                ms_per_step=round(total / steps * 1e3, 2), h2d_ms=round(t["h2d"] / steps * 1e3, 2),
                                run_ms=round(t["run"] / steps * 1e3, 2), d2h_ms=round(t["d2h"] / steps * 1e3, 2)),
                note="files in pinned host buffers (gck_host_register); value: gck_replay_into (H2D of file "
                     "groups overlapped with the replay of earlier groups, tuples D2H into a pinned array); "
                     "sequential: gck_ctx_load -> gck_ctx_run -> gck_ctx_fetch_into")


def keydir_merge(g, ctx, dist, n_files, reps=2):
    """N>1, after the timed replays: the exchange step of the sharded replay
    (gocask_amd.shard.merge_keydir) -- per-rank keydir with
    tombstones, hash partition, two RCCL all-to-alls, per-owner merge.  Not
    part of `value`; the slowest rank's seconds of the last of `reps` runs."""
    import torch

    from gocask_amd import shard

    base = shard.file_base(dist, n_files, device="cuda")
    for _ in range(reps):
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        n_live, ph = shard.merge_keydir(ctx, dist, base)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
    dev = "cpu" if dist.get_backend() == "gloo" else "cuda"
    v = torch.tensor([wall, ph["local"], ph["exchange"], ph["merge"]], dtype=torch.float64, device=dev)
    dist.all_reduce(v, op=dist.ReduceOp.MAX)
    c = torch.tensor([n_live, ph["sent_bytes"]], dtype=torch.float64, device=dev)
    dist.all_reduce(c, op=dist.ReduceOp.SUM)
    w, lo, ex, mg = (round(x * 1e3, 3) for x in v.tolist())
    return dict(ms=w, local_ms=lo, exchange_ms=ex, merge_ms=mg, live_entries=int(c[0].item()),
                exchanged_bytes=int(c[1].item()), global_status=ph["status"],
                note="global keydir over all ranks' files: keydir with tombstones per rank, key-hash partition, "
                     "RCCL all-to-all of entries + keys, per-owner last-shard-wins merge; max over ranks; "
                     "not part of value")


def replay_with_merge(ctx, dist, n_files, steps, my_bytes):
    """N>1: the path end to end -- every step replays the rank's shard and
    merges the global keydir over RCCL (shard.merge_keydir), timed together
    between barriers; the slowest rank's time, all ranks' bytes (the rate of
    `value` stops before the gather)."""
    import torch

    from gocask_amd import shard

    base = shard.file_base(dist, n_files, device="cuda")
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        ctx.run()
        shard.merge_keydir(ctx, dist, base)
    dist.barrier()
    torch.cuda.synchronize()
    elapsed, total = reduce_over_ranks(dist, time.perf_counter() - t0, my_bytes,
                                       "cpu" if dist.get_backend() == "gloo" else "cuda")
    return dict(value_with_merge=round(total * steps / elapsed / GiB, 2),
                ms_per_step_with_merge=round(elapsed / steps * 1e3, 3), steps=steps,
                note="every step: the replay of each rank's shard, then the keydir merge over RCCL "
                     "(all-to-all of key-hash partitions, last-shard-wins per owner); max over ranks")


def shard_config(cfg_name, rank):
    """A per-rank corpus for the configs that are not sharded (C1-C3, C5 at
    N > 1: rank r replays its own copy of the spec with seed + r)."""
    cfg = dict(CONFIGS[cfg_name])
    cfg["seed"] = cfg["seed"] + rank
    return cfg


def c4_spec(world, rank, files_per_rank=C4_FILES_PER_GPU, file_bytes=2 << 30):
    """(file ids, last_is_active, kw) of rank's C4 shard: the corpus has
    files_per_rank x world files, its key universe C4_KEYS_PER_FILE per 2 GiB
    file (scaled with file_bytes: --c4-file-mib shrinks the files of a
    rehearsal, not the spec)."""
    from gocask_amd import shard

    ids, last_active = shard.c4_file_ids(world, rank, files_per_rank)
    per_file = max(1, C4_KEYS_PER_FILE * file_bytes // (2 << 30))
    kw = dict(CONFIGS["c4"], key_universe=per_file * files_per_rank * world, max_file_size=file_bytes)
    return ids, last_active, kw


def encode_workload(ctx, cfg_name, world, rank, files_per_rank=C4_FILES_PER_GPU, file_bytes=2 << 30):
    """Encode this rank's files into its context.  C4: the rank's contiguous
    walk-order range of the one global corpus (no data-path collective: the
    files are independent)."""
    if cfg_name == "c4":
        ids, last_active, kw = c4_spec(world, rank, files_per_rank, file_bytes)
        return ctx.encode_files(ids, last_is_active=last_active, **kw)
    return ctx.encode(**shard_config(cfg_name, rank))


def launcher_cmd(n, argv, script=None):
    """The torch.distributed.run command that starts n rank processes of this
    script with the same arguments (one node; --standalone: the launcher's
    own c10d store picks a free port as it binds, on 127.0.0.1)."""
    return [sys.executable, "-m", "torch.distributed.run", "--standalone", "--nnodes=1", f"--nproc-per-node={n}",
            "--local-addr=127.0.0.1", script or os.path.abspath(__file__)] + list(argv)


def relaunch(n, argv):
    """--gpus N > 1 with no launcher around this process: run the N ranks as a
    child torch.distributed.run (nothing here has touched a GPU yet: only the
    argument parser ran), pass its output through (rank 0 prints the JSON
    line) and return its exit code.  A process that was itself started this
    way and still sees no WORLD_SIZE refuses to start another launcher."""
    import subprocess

    if os.environ.get("GCK_BENCH_LAUNCHED"):
        sys.exit("bench.py: started by bench.py's own launcher but no WORLD_SIZE: refusing a nested relaunch")
    env = dict(os.environ, GCK_BENCH_LAUNCHED="1")
    return subprocess.run(launcher_cmd(n, argv), env=env).returncode


def transport_label(devs):
    """What the library's keydir exchange crosses for contexts on devs."""
    if len(devs) == 1:
        return "RCCL self send/receive (one device: no xGMI link crossed)"
    if len(set(devs)) < len(devs):
        return "device copies (loopback)"
    return "RCCL over xGMI"


def lib_multi(args):
    """--lib-multi (see the module docstring): one process, one context per
    device, the library's own exchange + merge timed.  Prints one JSON line.
    One host thread per device, started once (a pool), so no timed step pays
    a thread's start-up."""
    from concurrent.futures import ThreadPoolExecutor

    import torch

    import gocask_amd as g

    n = args.gpus
    nvis = max(torch.cuda.device_count(), 1)
    devs = [d % nvis for d in range(n)]
    ctxs = [g.ReplayContext(device=dv, chunk_bytes=args.chunk_kib << 10) for dv in devs]
    infos = [None] * n
    pool = ThreadPoolExecutor(max_workers=n)

    def each(fn):
        list(pool.map(fn, range(n)))  # (re-raises a worker's exception)

    def enc(i):
        infos[i] = encode_workload(ctxs[i], "c4", n, i, args.c4_files_per_gpu, args.c4_file_mib << 20)

    each(enc)
    for _ in range(max(1, args.warmup)):
        each(lambda i: ctxs[i].run())
    for dv in sorted(set(devs)):
        torch.cuda.synchronize(dv)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        each(lambda i: ctxs[i].run())
    elapsed = time.perf_counter() - t0
    nbytes = sum(c.stats()["bytes"] for c in ctxs)
    merges = []
    for _ in range(2):
        t1 = time.perf_counter()
        _, st = g.multi_keydir(ctxs, fetch=False)
        merges.append((time.perf_counter() - t1, st))
    wall, st = merges[-1]
    # the path end to end: every step replays all shards and gathers the
    # global keydir (north_star: per-GPU fragments gathered over RCCL)
    t2 = time.perf_counter()
    for _ in range(args.steps):
        each(lambda i: ctxs[i].run())
        g.multi_keydir(ctxs, fetch=False)
    elapsed_m = time.perf_counter() - t2
    pool.shutdown()
    out = {
        "metric": "device-resident data-file GiB/s CRC-verified+header-decoded, 1 GPU (+2/4/8)",
        "value": round(nbytes * args.steps / elapsed / GiB, 2),
        "unit": "GiB/s",
        "n_gpus": n,
        "steps": args.steps,
        "mode": "lib-multi: one process, a context per device, replays from one host thread each",
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "value_with_merge": round(nbytes * args.steps / elapsed_m / GiB, 2),
        "ms_per_step_with_merge": round(elapsed_m / args.steps * 1e3, 3),
        "devices": devs,
        "keydir_merge_lib": dict(ms=round(wall * 1e3, 3), **{k + "_ms": round(v, 3) for k, v in st["ms"].items()},
                                 live_entries=st["n_live"], global_status=st["status"],
                                 transport=transport_label(devs),
                                 note="gck_ctx_multi_keydir: per device the keydir with tombstones packed over the "
                                      "owners, partitions exchanged in one RCCL group, per-owner merge (the library's "
                                      "own path behind gck_replay_multi); last of 2 runs; not part of value"),
    }
    print(json.dumps(out), flush=True)
    for c in ctxs:
        c.close()
    return 0


def lib_multi_child(args):
    """Rank 0 of an N>1 run, after every rank has released its GPU: the
    --lib-multi measurement as a child process (its own RCCL communicators
    over all N devices).  Returns its keydir_merge_lib (or the failure)."""
    import subprocess

    cmd = [sys.executable, os.path.abspath(__file__), "--gpus", str(args.gpus), "--lib-multi", "--steps", "2",
           "--warmup", "1", "--c4-files-per-gpu", str(args.c4_files_per_gpu), "--c4-file-mib", str(args.c4_file_mib),
           "--chunk-kib", str(args.chunk_kib)]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE",
                                                          "GROUP_RANK", "ROLE_RANK", "TORCHELASTIC_RUN_ID")}
    try:
        p = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env)
    except subprocess.TimeoutExpired:
        return dict(error="timeout after 240 s")
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    if p.returncode or not lines:
        return dict(error=f"rc {p.returncode}: {p.stderr[-400:]}")
    d = json.loads(lines[-1])
    return dict(d["keydir_merge_lib"], replay_gibs=d["value"], replay_ms_per_step=d["ms_per_step"],
                value_with_merge=d["value_with_merge"], ms_per_step_with_merge=d["ms_per_step_with_merge"])


def reduce_over_ranks(dist, elapsed, nbytes, device):
    """Whole-job timing: the slowest rank's time and the bytes of all ranks."""
    if dist is None:
        return elapsed, float(nbytes)
    import torch

    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    b = torch.tensor([float(nbytes)], dtype=torch.float64, device=device)
    dist.all_reduce(b, op=dist.ReduceOp.SUM)
    return float(t.item()), float(b.item())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default=None, choices=sorted(CONFIGS),
                    help="workload (default: c3 at one GPU, c4 -- one corpus sharded over the GPUs -- at N > 1)")
    ap.add_argument("--chunk-kib", type=int, default=0)
    ap.add_argument("--cpu-sample-gib", type=float, default=2.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--keydir", action="store_true", help="also time the device keydir (gck_ctx_keydir)")
    ap.add_argument("--no-merge", action="store_true",
                    help="N>1: skip the keydir merge across ranks that follows the timed replays")
    ap.add_argument("--spec-kib", type=int, default=0, help="speculation window per chunk (KiB, 0: default)")
    ap.add_argument("--chunk-cap", type=int, default=0, help="record slots staged per chunk (0: default)")
    ap.add_argument("--merge", action="store_true",
                    help="N=1: time the keydir merge too (a one-rank RCCL group)")
    ap.add_argument("--host-inclusive", type=int, default=0, metavar="K",
                    help="also time K host-in/host-out replays (pinned H2D + run + D2H of the tuples)")
    ap.add_argument("--c4-files-per-gpu", type=int, default=C4_FILES_PER_GPU,
                    help="C4: files per rank (16: BASELINE's C4; fewer only for rehearsals)")
    ap.add_argument("--c4-file-mib", type=int, default=2048,
                    help="C4: file size in MiB (2048: BASELINE's C4; smaller only for rehearsals)")
    ap.add_argument("--lib-multi", action="store_true",
                    help="one process, a context per device, the library's own keydir exchange (see above)")
    ap.add_argument("--no-lib-multi", action="store_true", help="N>1: skip the --lib-multi child at the end")
    args = ap.parse_args()
    if args.lib_multi:
        sys.exit(lib_multi(args))

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(relaunch(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world} rank processes")
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import torch

    dist = None
    # one GPU per rank; GCK_DIST_BACKEND=gloo rehearses N>1 with ranks sharing
    # fewer GPUs (device = local rank mod the GPUs present)
    device = local_rank % max(torch.cuda.device_count(), 1)
    backend = os.environ.get("GCK_DIST_BACKEND", "nccl")
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(device)
        dist.init_process_group(backend)
    elif torch.cuda.is_available():
        torch.cuda.set_device(device)

    import gocask_amd as g

    if args.config is None:
        args.config = "c3" if world == 1 else "c4"
    t_setup = time.perf_counter()
    ctx = g.ReplayContext(device=device, chunk_bytes=args.chunk_kib << 10, spec_window=args.spec_kib << 10,
                          chunk_cap=args.chunk_cap)
    info = encode_workload(ctx, args.config, world, rank, args.c4_files_per_gpu, args.c4_file_mib << 20)
    setup_s = time.perf_counter() - t_setup

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    for _ in range(args.warmup):
        ctx.run()
    barrier()
    s0 = ctx.stats()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ctx.run()
    barrier()
    elapsed = time.perf_counter() - t0
    st = ctx.stats()
    my_bytes = st["bytes"]
    # k_crc_rows' HIP-event time (recorded on its stream) averaged over the
    # timed steps themselves
    assert st["n_runs"] - s0["n_runs"] == args.steps
    crc_avg = (st["ms_crc_rows_sum"] - s0["ms_crc_rows_sum"]) / args.steps
    rank_elapsed = elapsed
    elapsed, total_bytes = reduce_over_ranks(dist, elapsed, my_bytes, "cpu" if backend == "gloo" else "cuda")
    # every rank's own figures (N > 1: the roofline of each rank's k_crc_rows)
    per_rank = [dict(rank=0, crc_rows_ms=crc_avg, step_ms=rank_elapsed / args.steps * 1e3, bytes=my_bytes)]
    if dist is not None:
        dev = "cpu" if backend == "gloo" else "cuda"
        mine = torch.tensor([crc_avg, rank_elapsed / args.steps * 1e3, float(my_bytes)], dtype=torch.float64,
                            device=dev)
        allr = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(allr, mine)
        per_rank = [dict(rank=r, crc_rows_ms=float(t[0].item()), step_ms=float(t[1].item()), bytes=int(t[2].item()))
                    for r, t in enumerate(allr)]
    # per-phase device times of a few more, untimed steps with an event between
    # every phase (the timed steps record only the events around k_crc_rows)
    phases_sum, n_phase = {}, 3
    ctx.phase_timing(True)
    for _ in range(n_phase):
        ctx.run()
        stp = ctx.stats()
        for k, v in stp["ms_phase"].items():
            phases_sum[k] = phases_sum.get(k, 0.0) + v
    ctx.phase_timing(False)
    merge = None
    if dist is None and args.merge:
        import socket

        import torch.distributed as dist1

        with socket.socket() as so:
            so.bind(("127.0.0.1", 0))
            port = so.getsockname()[1]
        dist1.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
        merge = keydir_merge(g, ctx, dist1, info["n_files"])
        dist1.destroy_process_group()
    elif dist is not None and not args.no_merge:
        merge = keydir_merge(g, ctx, dist, info["n_files"])
        merge["with_replay"] = replay_with_merge(ctx, dist, info["n_files"], args.steps, my_bytes)
    stream_gbs = rows_gbs = None
    if rank == 0:
        _, stream_gbs = ctx.stream_read_ceiling(5)
        # the balanced stream ceiling over k_crc_rows' rows (its loads, whole
        # 64-row blocks, half static and half from per-XCD queues, no
        # compute; core.stream_rows_ceiling), with the spread of its
        # wavefronts' end times from their clock stamps
        import numpy as np
        rows_end = None
        try:
            _, rows_gbs = ctx.stream_rows_ceiling(5, stamp=True)
            stamps, _ = ctx.clock_stamps()
            w = 4 * torch.cuda.get_device_properties(0).multi_processor_count
            s = stamps[:w].astype(np.float64)
            ok = (s[:, 1] > 0) & (s[:, 3] > s[:, 1])
            end = (s[ok, 3] - s[ok, 1].min()) / 100.0  # us (real time at 100 MHz)
            rows_end = [round(float(np.median(end)), 1), round(float(end.max()), 1)] if ok.any() else None
        except (AttributeError, RuntimeError):  # (an older build's diag library, in an A/B: no such probe)
            rows_gbs = None
    if rank == 0:
        ms_step = elapsed / args.steps * 1e3
        value = total_bytes * args.steps / elapsed / GiB
        launches = 1
        achieved = my_bytes / (crc_avg * 1e-3) / 1e9
        traffic = None
        tf = os.path.join(ROOT, "profiles", f"traffic_{args.config}.json")
        rehearsal = args.config == "c4" and (args.c4_file_mib != 2048 or args.c4_files_per_gpu != C4_FILES_PER_GPU)
        if os.path.exists(tf) and not rehearsal:
            traffic = json.load(open(tf)).get("crc_rows_hbm_bytes_per_launch")
        out = {
            "metric": "device-resident data-file GiB/s CRC-verified+header-decoded, 1 GPU (+2/4/8)",
            "value": round(value, 2),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (device-encoded GoCask records, DESIGN.md Corpus)",
            "config": {
                "workload": DESCR[args.config].format(n=args.c4_files_per_gpu * world, g=world)
                + (f" ({args.c4_file_mib} MiB files: a rehearsal, not BASELINE's C4)"
                   if args.config == "c4" and (args.c4_file_mib != 2048 or args.c4_files_per_gpu != C4_FILES_PER_GPU)
                   else "")
                + (" per GPU" if world > 1 and args.config != "c4" else ""),
                "bytes_per_gpu": my_bytes,
                "records_per_gpu": st["n_recs"],
                "files_per_gpu": info["n_files"],
                "crc_rejects": st["n_crc_fail"],
                "parallelism": f"files sharded over {world} GPU(s) in contiguous walk-order ranges, no data-path collective"
                               + ("; keydir merge over RCCL all-to-all after the timed replays" if world > 1 else ""),
            },
            "roofline": {
                "bound": "hbm",
                "kernel": "k_crc_rows",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "crc_rows_ms": round(crc_avg, 4),
                "launches_per_step": launches,
                "algorithmic_bytes_per_launch": round(my_bytes / launches),
                "note": "achieved = data-file bytes / HIP-event time of the k_crc_rows launch of a step, "
                        "averaged over the timed steps (one launch per step over all files)",
                "stream_read_gbs": round(stream_gbs, 1),
                "frac_of_stream_read": round(achieved / stream_gbs, 4),
                "rows_ceiling_gbs": round(rows_gbs, 1) if rows_gbs else None,
                "frac_of_rows_ceiling": round(achieved / rows_gbs, 4) if rows_gbs else None,
                "rows_ceiling_wave_end_us": rows_end,
                "ceilings_note": "stream_read: a static grid-stride non-temporal read of the arena; rows: the same "
                                 "bytes with k_crc_rows' loads in 64-row blocks, half static and the rest from one "
                                 "queue per XCD, 4 wavefronts per CU with 3 rows in flight, no compute -- the fastest "
                                 "stream measured whose wavefronts end together (wave_end_us: median and last "
                                 "wavefront's end from their clock stamps); both right after the timed steps, HIP events",
            },
            "phase_ms": {k: round(v / n_phase, 4) for k, v in phases_sum.items()},
        }
        if world > 1:
            # each rank's k_crc_rows over its own shard (rank 0's is the line's achieved / frac)
            out["roofline"]["per_rank"] = [
                dict(rank=p["rank"], crc_rows_ms=round(p["crc_rows_ms"], 4), step_ms=round(p["step_ms"], 3),
                     bytes=p["bytes"], achieved=round(p["bytes"] / (p["crc_rows_ms"] * 1e-3) / 1e9, 1),
                     frac=round(p["bytes"] / (p["crc_rows_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4))
                for p in per_rank]
            fr = [p["frac"] for p in out["roofline"]["per_rank"]]
            out["roofline"]["frac_min_over_ranks"] = min(fr)
            out["roofline"]["frac_max_over_ranks"] = max(fr)
        if args.keydir:
            ctx.keydir()  # warm-up (allocations)
            ctx.phase_timing(True)
            ctx.run()  # a fresh run: its first keydir hashes every key
            fin_plain = ctx.stats()["ms_phase"]["finalize"]
            live, kd_ms = ctx.keydir()
            _, kd_again_ms = ctx.keydir(fetch=False)
            ctx.keydir_hash(True)  # the run's finalize hashes the keys instead
            ctx.run()
            fin_hash = ctx.stats()["ms_phase"]["finalize"]
            _, kd_hashed_ms = ctx.keydir(fetch=False)
            ctx.keydir_hash(False)
            ctx.phase_timing(False)
            out["keydir"] = dict(ms=round(kd_ms, 3), live_entries=len(live), records=st["n_recs"],
                                 rebuild_ms=round(kd_again_ms, 3), after_finalize_hash_ms=round(kd_hashed_ms, 3),
                                 finalize_ms_plain=round(fin_plain, 4), finalize_ms_hashing=round(fin_hash, 4),
                                 note="gck_ctx_keydir, the first after a run (row f1): last record per key, Puts "
                                      "kept; rebuild_ms = a second keydir of the same run (its table kept: marking and compaction only); "
                                      "after_finalize_hash_ms = the keydir after a run whose finalize hashed the keys "
                                      "and inserted them into the keydir table (gck_ctx_keydir_hash; what GCK_OPT_LIVE "
                                      "runs), which costs finalize the difference shown; "
                                      "not part of value")
            ctx.scrub_keydir()  # warm-up
            _, _, bad, sc_ms = ctx.scrub_keydir()
            vbytes = int(live["value_size"].sum(dtype="u8"))
            out["scrub"] = dict(ms=round(sc_ms, 3), entries=len(live), value_bytes=vbytes, crc_rejects=bad,
                                gbs=round(vbytes / (sc_ms * 1e-3) / 1e9, 1),
                                note="gck_ctx_scrub_keydir (row f3): Get of every live key on the device -- "
                                     "value at (File, ValuePos) re-read and CRC-checked; not part of value")
        if merge is not None:
            out["keydir_merge"] = merge
            if "with_replay" in merge:
                # the path end to end (replay + gather), beside `value` (replay only)
                out["value_with_merge"] = merge["with_replay"]["value_with_merge"]
        if args.host_inclusive:
            out["host_inclusive"] = host_inclusive(g, ctx, info, args.host_inclusive)
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(args.config, int(args.cpu_sample_gib * GiB))
        lib_multi_pending = world > 1 and not args.no_lib_multi
        if args.verbose:
            out["setup_s"] = round(setup_s, 2)
            out["fixups"] = st["n_fixups"]
            out["overflow_chunks"] = st["n_overflow"]
    ctx.close()
    if dist is not None:
        dist.barrier()  # every rank's context freed before the child takes the GPUs
        dist.destroy_process_group()
    if rank == 0:
        if lib_multi_pending:
            out["keydir_merge_lib"] = lib_multi_child(args)
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
