"""Bounded-memory host-in/host-out replay (row f2): gck_replay /
gck_replay_into with a resident-bytes budget (gck_opts.max_resident) smaller
than the database.  The files are cut into groups after files that reset
lastOffset, and a ring of device contexts holds only a few groups at a time:
the reference replays any database size (core/db.go:110-143; data files
default to 10 GiB, db.go:45-48), so Open must not fail for want of HBM.
Results must equal the oracle's whatever the ring size."""
import numpy as np
import pytest

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


def _corpus(orc, seed=91, n_files=12, fsize=2 << 20, active=None):
    files, names = orc.gen_corpus(seed=seed, val_fixed=0, key_min=8, key_max=24, key_universe=3000,
                                  tomb_permille=30, flip_permille=20, max_file_size=fsize, n_files=n_files)
    walk = sorted(range(len(files)), key=lambda i: names[i])
    wf = [files[i] for i in walk]
    reset = [True] * len(wf)
    reset[len(wf) - 1 if active is None else active] = False
    return wf, reset


@pytest.mark.parametrize("budget", [8 << 20, 12 << 20, 1 << 20])
def test_ring_equals_oracle(g, orc, budget):
    wf, reset = _corpus(orc, active=4)  # the active file mid-way: its lastOffset carries into file 5
    want, wst = orc.replay(wf, reset)
    got, gst = g.replay(wf, reset, max_resident=budget)
    # groups of >= budget / 3 bytes (cut after resetting files); as many
    # resident at once as the budget holds of the largest
    assert gst["n_groups"] >= 4 and 1 <= gst["n_resident"] < gst["n_groups"], gst
    assert gst["n_resident"] == (1 if budget < (2 << 20) else 2)
    _same(got, gst, want, wst)
    # into caller memory: pageable (DMA copies) and pinned (k_push_recs)
    recs = np.zeros(len(want) + 5, dtype=g.REC_DTYPE)
    st = g.replay_into(wf, recs, reset, max_resident=budget)
    _same(recs[:st["n_recs"]], st, want, wst)
    g.host_register(recs)
    try:
        recs[:] = 0
        st = g.replay_into(wf, recs, reset, max_resident=budget)
        _same(recs[:st["n_recs"]], st, want, wst)
    finally:
        g.host_unregister(recs)
    small = np.zeros(10, dtype=g.REC_DTYPE)
    with pytest.raises(g._lib.GckError):
        g.replay_into(wf, small, reset, max_resident=budget)


def test_ring_startup_error_in_a_later_group(g, orc):
    wf, reset = _corpus(orc, seed=92)
    bad = np.frombuffer(orc_mod.entry(1, b"user", b"x" * 10) + orc_mod.entry(2, b"key", b"yy")[:-4], np.uint8)
    wf = wf[:7] + [bad] + wf[7:]
    reset = reset[:7] + [True] + reset[7:]
    want, wst = orc.replay(wf, reset)
    assert wst["status"] == 1 and wst["err_file"] == 7
    got, gst = g.replay(wf, reset, max_resident=6 << 20)
    assert gst["n_resident"] < gst["n_groups"]
    _same(got, gst, want, wst)
    assert gst["files_walked"] == 8


def test_ring_default_budget_keeps_everything_resident(g, orc):
    wf, reset = _corpus(orc, seed=93, n_files=6)
    want, wst = orc.replay(wf, reset)
    got, gst = g.replay(wf, reset)
    assert gst["n_resident"] == gst["n_groups"]
    _same(got, gst, want, wst)
