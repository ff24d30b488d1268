"""The cgo shim's calling pattern, in C, against the real
library (tests/shim/shim_test.c): files mmap'ed and pinned inside the Walk
callback while Disk.Walk still has them open (internal/fs/disk.go:128-144),
no files[0] when the walk finds no .csk file, gck_replay through
include/gocask_hip.h, records applied to a map in walk order.  Its keydir must
equal the reference tests' known answers (tests/golden/) and the oracle's."""
import os
import subprocess

import pytest

from golden_cases import load_case

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
SHIM = os.path.join(HERE, "shim", "build", "shim_test")


@pytest.fixture(scope="module")
def shim():
    import __graft_entry__

    __graft_entry__.build()
    subprocess.run(["make", "-s", "-C", os.path.join(HERE, "shim")], check=True)
    return SHIM


def run(shim, d, active=None, multi=False, mode="pinned", live=False):
    env = dict(os.environ, SHIM_MULTI="1" if multi else "0", SHIM_PIN="1" if mode == "pinned" else "0",
               SHIM_PATHS="1" if mode == "paths" else "0", SHIM_LIVE="1" if live else "0")
    p = subprocess.run([shim, str(d)] + ([active] if active else []), capture_output=True, text=True, timeout=120,
                       env=env)
    assert p.returncode == 0, p.stderr
    # (RCCL may print banner lines on stdout when the multi-GPU call loads it):
    # the result starts at the "status" line
    lines = p.stdout.splitlines()
    at = [i for i, ln in enumerate(lines) if ln.startswith("status ")]
    assert at, p.stdout[:2000]
    lines = lines[at[0]:]
    head = lines[0].split()
    st = dict(status=int(head[1]), last_offset=int(head[3]), keys=int(head[5]))
    kd = {}
    for ln in lines[1:]:
        k, crc, ts, pos, size, f = ln.split()
        kd[bytes.fromhex(k)] = dict(crc=int(crc), ts=int(ts), value_pos=int(pos), value_size=int(size), file=f)
    assert len(kd) == st["keys"]
    return st, kd


@pytest.mark.parametrize("name", ["existing_after_startup", "keys_in_order", "updated_values_across_files",
                                  "deleted_after_startup", "removed_keys", "datatxt_1000_puts", "crc_fail",
                                  "partial_write_desync"])
def test_shim_golden(shim, orc, tmp_path, name):
    meta, files, reset = load_case(name)
    assert sorted(meta["walk"]) == meta["walk"]  # a directory walks in this order too
    for w, f in zip(meta["walk"], files):
        (tmp_path / (w + ".csk")).write_bytes(f.tobytes())
    st, kd = run(shim, tmp_path, meta["active"])
    want, wst = orc.replay(files, reset)
    okd = orc.keydir(files, want, reset)
    assert st["status"] == wst["status"] and st["last_offset"] == wst["final_last_offset"]
    assert set(kd) == set(okd)
    for k, r in okd.items():
        e = kd[k]
        assert (e["crc"], e["ts"], e["value_pos"], e["value_size"]) == (
            int(r["crc"]), int(r["ts"]), int(r["value_pos"]), int(r["value_size"]))
        assert e["file"] == meta["walk"][int(r["file"])]
    if meta["status"] != "unexpected_eof":  # the reference tests' own answers
        assert set(kd) == {k.encode() for k in meta["expect"]}
        for k, x in meta["expect"].items():
            if "file" in x:
                assert kd[k.encode()]["file"] == x["file"]
        for k, x in meta.get("derived", {}).items():
            if isinstance(x, dict) and not k.startswith("_") and "value_pos" in x:
                assert kd[k.encode()]["value_pos"] == x["value_pos"], k


def test_shim_no_data_files(shim, tmp_path):
    # only a non-.csk entry: Disk.Open picks it as the active file, the walk
    # finds nothing; the shim must not index files[0]
    (tmp_path / "foo.txt").write_bytes(b"not a data file")
    st, kd = run(shim, tmp_path)
    assert st == dict(status=0, last_offset=0, keys=0) and kd == {}


def test_shim_disk_layout(shim, orc, tmp_path):
    # rotated data_<n>_<unix>.csk files, foo.txt, a nested directory; Disk.Open's
    # active file (the lexically last entry, "foo") never matches, so every
    # file resets lastOffset
    files, names = orc.gen_corpus(seed=23, val_fixed=0, key_min=8, key_max=16, key_universe=300, tomb_permille=40,
                                  flip_permille=20, max_file_size=1 << 16, n_files=10)
    (tmp_path / "a_sub").mkdir()
    nested = orc.entry(5, b"nested", b"v1") + orc.tombstone(6, b"k0000001")
    (tmp_path / "a_sub" / "data_9_1.csk").write_bytes(nested)
    for f, n in zip(files, names):
        (tmp_path / (n + ".csk")).write_bytes(f.tobytes())
    (tmp_path / "foo.txt").write_bytes(b"x")
    st, kd = run(shim, tmp_path)
    import numpy as np

    walk = ["data_9_1"] + sorted(names)
    wf = [np.frombuffer(nested, np.uint8)] + [files[names.index(n)] for n in sorted(names)]
    want, wst = orc.replay(wf, [True] * len(wf))
    okd = orc.keydir(wf, want, [True] * len(wf))
    assert st["status"] == 0 and st["last_offset"] == wst["final_last_offset"] == 0
    assert set(kd) == set(okd)
    for k, r in okd.items():
        assert kd[k]["value_pos"] == int(r["value_pos"]) and kd[k]["file"] == walk[int(r["file"])]


@pytest.mark.parametrize("name", ["existing_after_startup", "keys_in_order", "updated_values_across_files",
                                  "deleted_after_startup", "datatxt_1000_puts", "partial_write_desync"])
def test_shim_multi_gpu_call_same_keydir(shim, orc, tmp_path, name):
    """The shim's several-GPU call (gck_replay_multi, RCCL inside the library;
    one device here) gives the keydir and status of the single-GPU call."""
    meta, files, reset = load_case(name)
    for w, f in zip(meta["walk"], files):
        (tmp_path / (w + ".csk")).write_bytes(f.tobytes())
    one = run(shim, tmp_path, meta["active"])
    many = run(shim, tmp_path, meta["active"], multi=True)
    assert one == many


@pytest.mark.parametrize("name", ["existing_after_startup", "keys_in_order", "updated_values_across_files",
                                  "datatxt_1000_puts", "crc_fail", "partial_write_desync"])
def test_shim_pageable_and_by_path_same_keydir(shim, orc, tmp_path, name):
    """Open without pinning: the mappings staged by the library (SHIM_PIN=0),
    or the files named by path (gck_replay_paths, SHIM_PATHS=1), give the
    keydir and status of the pinned call."""
    meta, files, reset = load_case(name)
    for w, f in zip(meta["walk"], files):
        (tmp_path / (w + ".csk")).write_bytes(f.tobytes())
    pinned = run(shim, tmp_path, meta["active"])
    assert run(shim, tmp_path, meta["active"], mode="pageable") == pinned
    assert run(shim, tmp_path, meta["active"], mode="paths") == pinned
    assert run(shim, tmp_path, meta["active"], mode="paths", multi=True) == pinned


@pytest.mark.parametrize("name", ["existing_after_startup", "keys_in_order", "updated_values_across_files",
                                  "deleted_after_startup", "removed_keys", "datatxt_1000_puts", "crc_fail",
                                  "partial_write_desync"])
def test_shim_live_keydir_same_keydir(shim, orc, tmp_path, name):
    """GCK_OPT_LIVE on the single-GPU drop-in call (SHIM_LIVE=1): the live
    keydir comes back instead of every record, pinned and by path, and the
    shim's map equals the records mode's."""
    meta, files, reset = load_case(name)
    for w, f in zip(meta["walk"], files):
        (tmp_path / (w + ".csk")).write_bytes(f.tobytes())
    pinned = run(shim, tmp_path, meta["active"])
    assert run(shim, tmp_path, meta["active"], live=True) == pinned
    assert run(shim, tmp_path, meta["active"], mode="paths", live=True) == pinned


def test_shim_timing_mode_fills_the_map(shim, orc, tmp_path):
    """SHIM_TIME=1 (tools/shim_c3.py): the Open as the shim pays it, map fill
    included, in both modes; the map holds the oracle keydir's size."""
    import json

    files, names = orc.gen_corpus(seed=41, val_fixed=0, key_min=8, key_max=16, key_universe=500, tomb_permille=80,
                                  max_file_size=1 << 18, n_files=4)
    for f, n in zip(files, names):
        (tmp_path / (n + ".csk")).write_bytes(f.tobytes())
    walk = sorted(names)
    wf = [files[names.index(n)] for n in walk]
    reset = [i + 1 < len(wf) for i in range(len(wf))]
    want, _ = orc.replay(wf, reset)
    n_live = len(orc.keydir(wf, want, reset))
    for live in ("0", "1"):
        env = dict(os.environ, SHIM_TIME="1", SHIM_PATHS="1", SHIM_LIVE=live)
        p = subprocess.run([shim, str(tmp_path)], capture_output=True, text=True, timeout=120, env=env)
        assert p.returncode == 0, p.stderr
        d = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
        assert d["map_entries"] == n_live and d["live"] == int(live)
        assert d["records"] == (n_live if live == "1" else len(want))
