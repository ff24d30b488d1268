"""gck_replay_multi's N-owner orchestration on the one-GPU box: N logical
shards on device 0 (libgocask_diag.so's loopback entry), the partitions moved
by device copies instead of RCCL.  Everything else is the N-GPU call's code:
the shard plan, each shard's ring replay with a keydir pack per file group, the
global outcome, the receive layout (owner p, source i) and the per-owner
merges.  The result must be the oracle's global keydir (keyDir.set / unset over
every file in walk order, /root/reference/core/keydir.go:22-49) with the
reference's status (/root/reference/core/db.go:110-138)."""
import os

import numpy as np
import pytest

from golden_cases import case_names, load_case
from test_gpu_multi import _check, _keys_of

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def g():
    import __graft_entry__

    __graft_entry__.build()
    import gocask_amd

    assert gocask_amd.device_count() > 0, "no GPU visible"
    return gocask_amd


def _walk(orc, **kw):
    files, names = orc.gen_corpus(**kw)
    order = sorted(range(len(files)), key=lambda i: names[i])
    return [files[i] for i in order]


@pytest.mark.parametrize("nshards", [2, 3, 4])
@pytest.mark.parametrize("name", case_names())
def test_loopback_golden(g, orc, name, nshards):
    _, files, reset = load_case(name)
    want, wst = orc.replay(files, reset)
    got, gst = g.replay_multi_loopback(files, reset, nshards=nshards)
    _check(files, got, gst, want, wst)


@pytest.mark.parametrize("nshards", [2, 4])
def test_loopback_keys_in_order_carry(g, orc, nshards):
    # core/db_test.go:428-471: foobar (data01) has ValuePos 66
    meta, files, reset = load_case("keys_in_order")
    got, gst = g.replay_multi_loopback(files, reset, nshards=nshards)
    want, wst = orc.replay(files, reset)
    _check(files, got, gst, want, wst)
    pos = {bytes(files[int(r["file"])][int(r["rec_off"]) + 16:int(r["rec_off"]) + 16 + int(r["key_len"])]):
           int(r["value_pos"]) for r in got}
    assert pos[b"foobar"] == 66 and gst["final_last_offset"] == meta["final_last_offset"]


@pytest.mark.parametrize("nshards,budget", [(2, 0), (3, 0), (4, 0), (3, 3 << 20), (4, 2 << 20)])
def test_loopback_cross_shard_overwrite_and_delete(g, orc, nshards, budget):
    """Twelve files over a small key universe: keys repeat across shards, a
    later shard's Put overwrites and its Delete hides an earlier shard's; with
    a budget every shard streams through a ring of several file groups (a
    source per group), so the merge sees many sources per owner."""
    wf = _walk(orc, seed=811, val_fixed=0, key_min=8, key_max=20, key_universe=900, tomb_permille=200,
               flip_permille=25, max_file_size=1 << 20, n_files=12)
    reset = [True] * len(wf)
    reset[-1] = False
    want, wst = orc.replay(wf, reset)
    got, gst = g.replay_multi_loopback(wf, reset, nshards=nshards, max_resident=budget)
    _check(wf, got, gst, want, wst)
    if budget:
        assert gst["n_groups"] > nshards  # several groups per shard went through the ring


def test_loopback_active_file_mid_walk(g, orc):
    """The active file (walked first, data_* sorts before data_<n>...) does
    not reset lastOffset; no cut may follow it, so its carry stays in a shard."""
    wf = _walk(orc, seed=812, val_fixed=0, key_min=8, key_max=16, key_universe=300, tomb_permille=100,
               max_file_size=1 << 18, n_files=8)
    reset = [True] * len(wf)
    reset[2] = False
    reset[5] = False
    want, wst = orc.replay(wf, reset)
    for n in (2, 3, 4):
        got, gst = g.replay_multi_loopback(wf, reset, nshards=n)
        _check(wf, got, gst, want, wst)


@pytest.mark.parametrize("where", [1, 4, 7])
def test_loopback_startup_error(g, orc, where):
    """A partial write in file `where` aborts the walk there: earlier shards and
    the failing shard's records before the error count, later shards nothing."""
    wf = _walk(orc, seed=813, val_fixed=0, key_min=8, key_max=16, key_universe=500, tomb_permille=120,
               max_file_size=1 << 17, n_files=8)
    _, bad, _ = load_case("partial_write_desync")
    wf = wf[:where] + [bad[0]] + wf[where:]
    reset = [True] * (len(wf) - 1) + [False]
    want, wst = orc.replay(wf, reset)
    assert wst["status"] == 1 and wst["err_file"] == where
    for n in (2, 3, 4):
        got, gst = g.replay_multi_loopback(wf, reset, nshards=n)
        _check(wf, got, gst, want, wst)
        got2, gst2 = g.replay_multi_loopback(wf, reset, nshards=n, max_resident=1 << 20)
        _check(wf, got2, gst2, want, wst)


@pytest.mark.parametrize("nshards", [2, 4])
def test_loopback_keys(g, orc, nshards):
    """GCK_OPT_KEYS: the live entries' key bytes, in the order of the records."""
    wf = _walk(orc, seed=814, val_fixed=0, key_min=8, key_max=24, key_universe=700, tomb_permille=100,
               max_file_size=1 << 19, n_files=6)
    reset = [True] * (len(wf) - 1) + [False]
    want, wst = orc.replay(wf, reset)
    got, gst = g.replay_multi_loopback(wf, reset, nshards=nshards, keys=True)
    _check(wf, got, gst, want, wst)
    assert np.array_equal(gst["keys"], _keys_of(wf, got))


def test_loopback_more_shards_than_cuts(g, orc):
    """Two files, four shards: two shards are empty (no cut allowed)."""
    _, files, reset = load_case("updated_values_across_files")
    want, wst = orc.replay(files, reset)
    got, gst = g.replay_multi_loopback(files, reset, nshards=4)
    _check(files, got, gst, want, wst)


def test_multi_one_device_rccl_self(g, orc):
    """GCK_MULTI_RCCL_SELF=1: on one device the library's RCCL path (a
    one-rank communicator, grouped self send / receive) carries the partition
    instead of a device copy; same keydir."""
    wf = _walk(orc, seed=815, val_fixed=0, key_min=8, key_max=16, key_universe=600, tomb_permille=150,
               flip_permille=20, max_file_size=1 << 19, n_files=5)
    reset = [True] * (len(wf) - 1) + [False]
    want, wst = orc.replay(wf, reset)
    os.environ["GCK_MULTI_RCCL_SELF"] = "1"
    try:
        got, gst = g.replay_multi(wf, reset, devices=[0])
    finally:
        del os.environ["GCK_MULTI_RCCL_SELF"]
    _check(wf, got, gst, want, wst)
