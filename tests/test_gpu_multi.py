"""gck_replay_multi: the sharded replay and the keydir merge behind one C-ABI
call (the drop-in Open of north_star on several GPUs).  On the
one-GPU box it runs with one device: the library's own RCCL communicator
(ncclCommInitAll) and grouped send / recv carry the partitions, and the
result must be the oracle's global keydir (keyDir.set / unset over every file
in walk order, core/keydir.go:22-49) with the reference's status."""
import numpy as np
import pytest

import oracle as orc_mod
from golden_cases import case_names, load_case

pytestmark = pytest.mark.gpu

FIELDS = ("rec_off", "file", "key_len", "value_pos", "value_size", "crc", "ts", "flags", "crc_calc")


@pytest.fixture(scope="module")
def g():
    import __graft_entry__

    __graft_entry__.build()
    import gocask_amd

    assert gocask_amd.device_count() > 0, "no GPU visible"
    return gocask_amd


def _check(files, got, gst, want, wst):
    for k in ("status", "files_walked", "final_last_offset"):
        assert gst[k] == wst[k], (k, gst, wst)
    if wst["status"]:
        assert (gst["err_file"], gst["err_off"]) == (wst["err_file"], wst["err_off"])
    kd = {}
    for r in want:  # the reference's keydir: records in walk order, deletes applied
        o = int(r["rec_off"]) + 16
        key = bytes(files[int(r["file"])][o:o + int(r["key_len"])])
        if int(r["flags"]) & 1:
            kd.pop(key, None)
        else:
            kd[key] = r
    assert len(got) == len(kd)
    seen = set()
    for r in got:
        o = int(r["rec_off"]) + 16
        key = bytes(files[int(r["file"])][o:o + int(r["key_len"])])
        assert key in kd and key not in seen
        seen.add(key)
        for f in FIELDS:
            assert r[f] == kd[key][f], (key, f)
    n_rej = int(((want["flags"] & 2) == 0).sum())
    assert gst["n_crc_fail"] == n_rej


@pytest.mark.parametrize("name", case_names())
def test_multi_one_device_golden(g, orc, name):
    _, files, reset = load_case(name)
    want, wst = orc.replay(files, reset)
    got, gst = g.replay_multi(files, reset, devices=[0])
    _check(files, got, gst, want, wst)


def test_multi_keys_in_order_carry(g, orc):
    # core/db_test.go:428-471: foobar in data01 has ValuePos 66 (the active
    # "data", walked first, does not reset lastOffset)
    meta, files, reset = load_case("keys_in_order")
    got, gst = g.replay_multi(files, reset, devices=[0])
    want, wst = orc.replay(files, reset)
    _check(files, got, gst, want, wst)
    pos = {bytes(files[int(r["file"])][int(r["rec_off"]) + 16:int(r["rec_off"]) + 16 + int(r["key_len"])]):
           int(r["value_pos"]) for r in got}
    assert pos[b"foobar"] == 66 and gst["final_last_offset"] == meta["final_last_offset"]


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_multi_random_with_deletes_and_flips(g, orc, seed):
    files, names = orc.gen_corpus(seed=600 + seed, val_fixed=0, key_min=8, key_max=24, key_universe=2000,
                                  tomb_permille=150, flip_permille=20, max_file_size=1 << 20, n_files=5)
    walk = sorted(range(len(files)), key=lambda i: names[i])
    wf = [files[i] for i in walk]
    reset = [i + 1 < len(wf) for i in range(len(wf))]
    want, wst = orc.replay(wf, reset)
    got, gst = g.replay_multi(wf, reset, devices=[0])
    _check(wf, got, gst, want, wst)


def test_multi_startup_error(g, orc):
    files, names = orc.gen_corpus(seed=77, val_fixed=0, key_min=8, key_max=16, key_universe=400,
                                  tomb_permille=150, max_file_size=1 << 17, n_files=4)
    walk = sorted(range(len(files)), key=lambda i: names[i])
    wf = [files[i] for i in walk]
    _, bad, _ = load_case("partial_write_desync")
    wf = wf[:2] + [bad[0]] + wf[2:]
    reset = [True] * (len(wf) - 1) + [False]
    want, wst = orc.replay(wf, reset)
    assert wst["status"] == 1 and wst["err_file"] == 2
    got, gst = g.replay_multi(wf, reset, devices=[0])
    _check(wf, got, gst, want, wst)


def test_multi_rejects_a_device_twice(g):
    files = [np.frombuffer(orc_mod.entry(1, b"k", b"v"), np.uint8)]
    with pytest.raises(g._lib.GckError):
        g.replay_multi(files, [False], devices=[0, 0])


def _keys_of(files, got):
    out = bytearray()
    for r in got:
        o = int(r["rec_off"]) + 16
        out += bytes(np.asarray(files[int(r["file"])], dtype=np.uint8)[o:o + int(r["key_len"])])
    return np.frombuffer(bytes(out), np.uint8)


@pytest.mark.parametrize("name", ["keys_in_order", "updated_values_across_files", "deleted_after_startup",
                                  "datatxt_1000_puts", "partial_write_desync"])
def test_multi_by_path_with_keys(g, orc, tmp_path, name):
    """gck_replay_multi_paths (the library reads the files) and GCK_OPT_KEYS
    (the live entries' key bytes in the order of the records): the same
    keydir as from memory, and the keys those records point at."""
    _, files, reset = load_case(name)
    paths = []
    for i, f in enumerate(files):
        p = tmp_path / f"{i:03d}.csk"
        p.write_bytes(f.tobytes())
        paths.append(str(p))
    want, wst = orc.replay(files, reset)
    got, gst = g.replay_multi_paths(paths, reset, devices=[0], keys=True)
    _check(files, got, gst, want, wst)
    assert np.array_equal(gst["keys"], _keys_of(files, got))
    got2, gst2 = g.replay_multi(files, reset, devices=[0], keys=True)
    assert np.array_equal(got2, got) and np.array_equal(gst2["keys"], gst["keys"])
