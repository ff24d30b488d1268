"""Open by path (row f2): gck_replay_paths reads the data files itself --
pread into page-locked staging buffers on host threads, streamed to the device
file group by file group -- so a caller needs neither mmap nor
gck_host_register (the cost of pinning a whole database).  The
same staging copier now carries gck_replay's pageable (unregistered) memory.
Results must equal the oracle's (core/db.go:110-178) for any ring size,
thread count and staging-chunk split."""
import os

import numpy as np
import pytest

import golden_cases
import oracle as orc_mod

pytestmark = pytest.mark.gpu

FIELDS = ("rec_off", "file", "key_len", "value_pos", "value_size", "crc", "ts", "flags", "crc_calc")


@pytest.fixture(scope="module")
def g():
    import __graft_entry__

    __graft_entry__.build()
    import gocask_amd

    assert gocask_amd.device_count() > 0, "no GPU visible"
    return gocask_amd


def _same(got, gst, want, wst):
    for k in ("status", "err_file", "err_off", "files_walked", "final_last_offset"):
        if k in ("err_file", "err_off") and not wst["status"]:
            continue
        assert gst[k] == wst[k], (k, gst, wst)
    assert len(got) == len(want)
    for f in FIELDS:
        assert np.array_equal(got[f], want[f]), f


def _write(tmp_path, files, tag="f"):
    paths = []
    for i, f in enumerate(files):
        p = tmp_path / f"{tag}_{i:04d}.csk"
        p.write_bytes(bytes(np.asarray(f, dtype=np.uint8)))
        paths.append(str(p))
    return paths


def _corpus(orc, seed=93, n_files=12, fsize=2 << 20, active=4):
    files, names = orc.gen_corpus(seed=seed, val_fixed=0, key_min=8, key_max=24, key_universe=3000,
                                  tomb_permille=30, flip_permille=20, max_file_size=fsize, n_files=n_files)
    walk = sorted(range(len(files)), key=lambda i: names[i])
    wf = [files[i] for i in walk]
    reset = [True] * len(wf)
    reset[active] = False  # the active file mid-way: its lastOffset carries on
    return wf, reset


@pytest.mark.parametrize("budget", [0, 12 << 20, 1 << 20])
@pytest.mark.parametrize("threads", ["1", "3"])
def test_paths_equal_oracle(g, orc, tmp_path, monkeypatch, budget, threads):
    monkeypatch.setenv("GCK_COPY_THREADS", threads)
    wf, reset = _corpus(orc)
    want, wst = orc.replay(wf, reset)
    got, gst = g.replay_paths(_write(tmp_path, wf), reset, max_resident=budget)
    _same(got, gst, want, wst)
    if budget:
        assert 1 <= gst["n_resident"] < gst["n_groups"], gst
    # the same files from pageable memory (the staging copier's memcpy path)
    got, gst = g.replay(wf, reset, max_resident=budget)
    _same(got, gst, want, wst)


@pytest.mark.parametrize("name", golden_cases.case_names())
def test_paths_golden(g, orc, tmp_path, name):
    meta, files, reset = golden_cases.load_case(name)
    want, wst = orc.replay(files, reset)
    got, gst = g.replay_paths(_write(tmp_path, files), reset)
    _same(got, gst, want, wst)


def test_paths_files_larger_than_a_staging_chunk(g, orc, tmp_path, monkeypatch):
    # 32 MiB staging chunks: files of 70 and 33 MiB cross chunk edges, and the
    # chunks of one file land in different buffers out of order
    monkeypatch.setenv("GCK_COPY_THREADS", "4")
    wf, reset = _corpus(orc, seed=94, n_files=3, fsize=70 << 20, active=2)
    assert max(len(f) for f in wf) > (64 << 20)
    want, wst = orc.replay(wf, reset)
    got, gst = g.replay_paths(_write(tmp_path, wf), reset)
    _same(got, gst, want, wst)


def test_paths_staging_by_hostmalloc(g, orc, tmp_path):
    # The staging buffers are registered huge-page memory by default and
    # hipHostMalloc memory when registration fails; GCK_STAGE_HOSTMALLOC (read
    # once per process) forces the second kind, so a child process replays
    # with it and the parent compares with the oracle.
    import subprocess
    import sys

    wf, reset = _corpus(orc, seed=95, n_files=5, fsize=3 << 20, active=2)
    want, wst = orc.replay(wf, reset)
    paths = _write(tmp_path, wf)
    out = tmp_path / "got.npy"
    code = ("import sys, json, numpy as np; sys.path.insert(0, sys.argv[1]); import gocask_amd as g; "
            "got, st = g.replay_paths(json.loads(sys.argv[2]), json.loads(sys.argv[3])); "
            "np.save(sys.argv[4], got); print(json.dumps({k: int(v) for k, v in st.items() "
            "if isinstance(v, (int, np.integer))}))")
    import json

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, GCK_STAGE_HOSTMALLOC="1")
    p = subprocess.run([sys.executable, "-c", code, root, json.dumps(paths), json.dumps(reset), str(out)],
                       capture_output=True, text=True, timeout=300, env=env)
    assert p.returncode == 0, p.stderr[-2000:]
    gst = json.loads(p.stdout.strip().splitlines()[-1])
    _same(np.load(out), gst, want, wst)


def test_paths_startup_error_and_empty_files(g, orc, tmp_path):
    wf, reset = _corpus(orc, seed=95, n_files=6)
    bad = np.frombuffer(orc_mod.entry(1, b"user", b"x" * 10) + orc_mod.entry(2, b"key", b"yy")[:-4], np.uint8)
    empty = np.zeros(0, np.uint8)
    wf = wf[:2] + [empty] + wf[2:4] + [bad] + wf[4:]
    reset = reset[:2] + [True] + reset[2:4] + [True] + reset[4:]
    want, wst = orc.replay(wf, reset)
    assert wst["status"] != 0
    got, gst = g.replay_paths(_write(tmp_path, wf), reset, max_resident=4 << 20)
    _same(got, gst, want, wst)


def test_paths_missing_or_unreadable_file(g, tmp_path):
    with pytest.raises(g._lib.GckError) as e:
        g.replay_paths([str(tmp_path / "absent.csk")], [False])
    assert e.value.code == g._lib.GCK_EIO
    assert not os.path.exists(tmp_path / "absent.csk")
    # a directory named as a data file is not a regular file: GCK_EIO
    d = tmp_path / "adir.csk"
    d.mkdir()
    (d / "x").write_bytes(b"y" * 100)
    with pytest.raises(g._lib.GckError) as e:
        g.replay_paths([str(d)], [False])
    assert e.value.code == g._lib.GCK_EIO


def test_paths_more_files_than_descriptors(g, orc, tmp_path):
    """no descriptor is held per file across the call (the copier
    opens a file per chunk it reads), so a database with more data files than
    the soft RLIMIT_NOFILE left to the process still replays, as the
    reference's Walk opens one file at a time (internal/fs/disk.go:122-145)."""
    import resource

    wf, _ = _corpus(orc, seed=97, n_files=1, active=0)
    recs, _ = orc.replay(wf[:1], [True])
    ends = [int(o) for o in recs["rec_off"][1:40]]  # record boundaries: every file replays whole
    files = [wf[0][: ends[(i * 7) % len(ends)]] for i in range(160)]
    reset = [True] * 159 + [False]
    want, wst = orc.replay(files, reset)
    assert wst["status"] == 0 and len(want) > 160
    paths = _write(tmp_path, files)
    soft, hard = resource.getrlimit(resource.RLIMIT_NOFILE)
    open_now = len(os.listdir("/proc/self/fd"))
    lim = open_now + 48  # fewer free descriptors than files
    assert lim < len(files) + open_now
    resource.setrlimit(resource.RLIMIT_NOFILE, (min(lim, soft), hard))
    try:
        got, gst = g.replay_paths(paths, reset)
    finally:
        resource.setrlimit(resource.RLIMIT_NOFILE, (soft, hard))
    _same(got, gst, want, wst)


def _want_keys(files, want):
    """The oracle records' key bytes back to back (record i: key_len bytes at
    its header + 16; a tombstone's key is its value, core/db.go:151-155)."""
    out = bytearray()
    for r in want:
        f = np.asarray(files[int(r["file"])], dtype=np.uint8)
        o = int(r["rec_off"]) + 16
        out += bytes(f[o:o + int(r["key_len"])])
    return np.frombuffer(bytes(out), np.uint8)


@pytest.mark.parametrize("budget", [0, 1 << 20])
def test_keys_blob(g, orc, tmp_path, budget):
    # GCK_OPT_KEYS: a caller that never maps the files gets the key bytes with
    # the records (the Go map needs them), for every entry point
    wf, reset = _corpus(orc, seed=96)
    want, wst = orc.replay(wf, reset)
    wk = _want_keys(wf, want)
    got, gst = g.replay_paths(_write(tmp_path, wf), reset, max_resident=budget, keys=True)
    _same(got, gst, want, wst)
    assert np.array_equal(gst["keys"], wk)
    got, gst = g.replay(wf, reset, max_resident=budget, keys=True)
    assert np.array_equal(gst["keys"], wk)
    recs = np.zeros(len(want), dtype=g.REC_DTYPE)
    st = g.replay_into(wf, recs, reset, max_resident=budget, keys=True)
    _same(recs, st, want, wst)
    assert np.array_equal(st["keys"], wk)
    # without the flag: no blob
    _, gst = g.replay(wf, reset, max_resident=budget)
    assert "keys" not in gst


def test_keys_blob_with_startup_error(g, orc, tmp_path):
    # only the records the reference applies before the error, and their keys
    wf, reset = _corpus(orc, seed=97, n_files=5)
    bad = np.frombuffer(orc_mod.entry(1, b"user", b"x" * 10) + orc_mod.entry(2, b"key", b"yy")[:-4], np.uint8)
    wf = wf[:3] + [bad] + wf[3:]
    reset = reset[:3] + [True] + reset[3:]
    want, wst = orc.replay(wf, reset)
    assert wst["status"] != 0
    got, gst = g.replay_paths(_write(tmp_path, wf), reset, max_resident=2 << 20, keys=True)
    _same(got, gst, want, wst)
    assert np.array_equal(gst["keys"], _want_keys(wf, want))
