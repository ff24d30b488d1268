"""bench.py --gpus N: the scaling curve the driver asks for comes from one
command.  With no launcher around it (no WORLD_SIZE), bench.py starts the N
rank processes itself (a torch.distributed.run child) before it touches a
GPU and passes rank 0's JSON line through; under a launcher the world size must
equal --gpus.  The reference's Open is one call over every file
(/root/reference/db.go:29-59); the N-GPU line is the sharded form of it."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_launcher_cmd_shape():
    import bench

    cmd = bench.launcher_cmd(4, ["--gpus", "4", "--steps", "3"], script="/x/bench.py")
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd
    # the launcher's own store picks the port (no port chosen here and freed
    # before the launcher binds it) on 127.0.0.1
    assert "--standalone" in cmd and "--local-addr=127.0.0.1" in cmd
    assert not any(a.startswith("--master-port") for a in cmd)
    assert cmd[-4:] == ["/x/bench.py", "--gpus", "4", "--steps", "3"][-4:]
    assert cmd.index("/x/bench.py") > cmd.index("--local-addr=127.0.0.1")


def test_nested_relaunch_refused():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["GCK_BENCH_LAUNCHED"] = "1"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "nested relaunch" in r.stderr


def test_world_size_must_match_gpus():
    """Under a launcher, a world of 3 ranks with --gpus 2 is refused before any
    GPU work (the line would be mislabelled otherwise)."""
    env = dict(os.environ, WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert "WORLD_SIZE=3" in r.stderr


def test_c4_spec_rehearsal_scaling():
    """--c4-file-mib shrinks the files and the key universe with them; the
    default is BASELINE's C4 (2 GiB files, 312,500 key ids per file)."""
    import bench

    ids, last, kw = bench.c4_spec(8, 7)
    assert len(ids) == 16 and last and kw["max_file_size"] == 2 << 30
    assert kw["key_universe"] == 312_500 * 128
    ids, last, kw = bench.c4_spec(2, 0, files_per_rank=2, file_bytes=64 << 20)
    assert len(ids) == 2 and not last and kw["max_file_size"] == 64 << 20
    assert kw["key_universe"] == (312_500 * 64 // 2048) * 4


@pytest.mark.gpu
def test_bench_gpus2_launches_its_ranks():
    """`python bench.py --gpus 2` on the one-GPU box: two rank processes over
    gloo (GCK_DIST_BACKEND, both on cuda:0), a small C4 (2 files of 64 MiB per
    rank), the keydir merge after the timed replays; one JSON line with
    n_gpus 2 and both ranks' k_crc_rows figures."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["GCK_DIST_BACKEND"] = "gloo"
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
           "--c4-files-per-gpu", "2", "--c4-file-mib", "64"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]  # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 3 and d["scaling"] == "weak"
    assert d["config"]["files_per_gpu"] == 2
    pr = d["roofline"]["per_rank"]
    assert [p["rank"] for p in pr] == [0, 1]
    assert all(p["crc_rows_ms"] > 0 and p["bytes"] > 0 for p in pr)
    # whole-job value: both ranks' bytes over the slowest rank's time
    tot = sum(p["bytes"] for p in pr)
    assert abs(d["value"] - tot * d["steps"] / (d["ms_per_step"] * 1e-3 * d["steps"]) / (1 << 30)) < 0.02 * d["value"]
    assert d["roofline"]["traffic"] is None  # a rehearsal carries no C4 counter bytes
    km = d["keydir_merge"]
    assert km["global_status"]["status"] == 0 and km["live_entries"] > 0
    # the drop-in multi-GPU path's exchange (gck_ctx_multi_keydir, one
    # process; on one GPU the two shards' partitions move by device copies):
    # the same global keydir as the torch path's merge
    kl = d["keydir_merge_lib"]
    assert "error" not in kl, kl
    assert kl["live_entries"] == km["live_entries"] and kl["global_status"] == 0
    assert kl["transport"].startswith("device copies")
    # replay + gather timed together: slower than the replay alone, positive
    assert 0 < d["value_with_merge"] < d["value"]
    assert 0 < kl["value_with_merge"] < kl["replay_gibs"]


@pytest.mark.gpu
@pytest.mark.parametrize("n,self_rccl", [(1, True), (3, False)])
def test_bench_lib_multi(n, self_rccl):
    """`bench.py --gpus N --lib-multi`: one process, a context per device (on
    the one-GPU box: N=1 through the library's RCCL path as a self send /
    receive, N=3 as a loopback of three contexts on device 0), the library's
    keydir exchange + merge timed as keydir_merge_lib."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    if self_rccl:
        env["GCK_MULTI_RCCL_SELF"] = "1"
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--lib-multi", "--steps", "2",
           "--warmup", "1", "--c4-files-per-gpu", "2", "--c4-file-mib", "64"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert d["n_gpus"] == n and d["value"] > 0
    kl = d["keydir_merge_lib"]
    assert kl["live_entries"] > 0 and kl["global_status"] == 0 and kl["ms"] > 0
    assert kl["transport"] == ("RCCL self send/receive (one device: no xGMI link crossed)" if n == 1
                               else "device copies (loopback)")
    assert 0 < d["value_with_merge"] < d["value"]
