"""GCK_OPT_LIVE: the single-GPU drop-in replay returns the live keydir (the
device keydir of SURVEY.md §8f f1, built per file group and merged across
groups in walk order) instead of every record, so the shim's Go map takes
one insert per live key.  The result must be the oracle's keydir (keyDir.set
/ unset over every file in walk order, core/keydir.go:22-49) with the
reference's status, through gck_replay, gck_replay_paths and
gck_replay_into, with and without GCK_OPT_KEYS, for one group and for rings
of several groups (max_resident)."""
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


@pytest.mark.parametrize("name", case_names())
def test_live_golden(g, orc, name):
    _, files, reset = load_case(name)
    want, wst = orc.replay(files, reset)
    got, gst = g.replay(files, reset, live=True, keys=True)
    _check(files, got, gst, want, wst)
    assert np.array_equal(gst["keys"], _keys_of(files, got))


@pytest.mark.parametrize("name", ["keys_in_order", "updated_values_across_files", "deleted_after_startup",
                                  "datatxt_1000_puts", "partial_write_desync", "empty_db"])
def test_live_by_path(g, orc, tmp_path, name):
    _, files, reset = load_case(name)
    paths = []
    for i, f in enumerate(files):
        p = tmp_path / f"{i:03d}.csk"
        p.write_bytes(np.asarray(f, dtype=np.uint8).tobytes())
        paths.append(str(p))
    want, wst = orc.replay(files, reset)
    got, gst = g.replay_paths(paths, reset, live=True, keys=True)
    _check(files, got, gst, want, wst)
    assert np.array_equal(gst["keys"], _keys_of(files, got))


@pytest.mark.parametrize("seed,max_resident", [(1, 0), (2, 3 << 20), (3, 1 << 20)])
def test_live_random_rings(g, orc, seed, max_resident):
    """Deletes, overwrites and flipped values across 6 files; small
    max_resident budgets cut them into groups whose keydirs merge."""
    files, names = orc.gen_corpus(seed=900 + seed, val_fixed=0, key_min=8, key_max=24, key_universe=1500,
                                  tomb_permille=120, flip_permille=20, max_file_size=1 << 20, n_files=6)
    walk = sorted(range(len(files)), key=lambda i: names[i])
    wf = [files[i] for i in walk]
    reset = [i + 1 < len(wf) for i in range(len(wf))]
    want, wst = orc.replay(wf, reset)
    got, gst = g.replay(wf, reset, live=True, max_resident=max_resident)
    _check(wf, got, gst, want, wst)
    if max_resident:
        assert gst["n_groups"] > 1


def test_live_into_and_capacity(g, orc):
    files, names = orc.gen_corpus(seed=931, val_fixed=0, key_min=8, key_max=16, key_universe=300,
                                  tomb_permille=100, max_file_size=1 << 18, n_files=3)
    walk = sorted(range(len(files)), key=lambda i: names[i])
    wf = [files[i] for i in walk]
    reset = [i + 1 < len(wf) for i in range(len(wf))]
    want, wst = orc.replay(wf, reset)
    ref, _ = g.replay(wf, reset, live=True)
    recs = np.zeros(len(ref) + 5, dtype=g.REC_DTYPE)
    st = g.replay_into(wf, recs, reset, live=True)
    assert st["n_recs"] == len(ref)
    assert np.array_equal(recs[:len(ref)], ref)
    _check(wf, recs[:len(ref)], st, want, wst)
    small = np.zeros(max(1, len(ref) - 1), dtype=g.REC_DTYPE)
    with pytest.raises(g._lib.GckError):
        g.replay_into(wf, small, reset, live=True)


def test_live_startup_error_in_a_later_group(g, orc):
    files, names = orc.gen_corpus(seed=77, val_fixed=0, key_min=8, key_max=16, key_universe=400,
                                  tomb_permille=150, max_file_size=1 << 17, n_files=4)
    walk = sorted(range(len(files)), key=lambda i: names[i])
    wf = [files[i] for i in walk]
    _, bad, _ = load_case("partial_write_desync")
    wf = wf[:2] + [bad[0]] + wf[2:]
    reset = [True] * (len(wf) - 1) + [False]
    want, wst = orc.replay(wf, reset)
    assert wst["status"] == 1 and wst["err_file"] == 2
    got, gst = g.replay(wf, reset, live=True, max_resident=1 << 17)
    _check(wf, got, gst, want, wst)
