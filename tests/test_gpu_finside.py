"""k_finalize beside k_crc_rows.  The device path cuts the CRC
pass into row pieces on a CU-masked stream and finalizes each finished piece
on the other CUs; the last piece's finalize runs on the whole chip.  A record
belongs to the piece holding its last byte (its range comes from row_first),
so records that span piece boundaries, files that start or end inside a
piece, CRC rejects and startup errors must all come out as the oracle's.
Forced shapes (GCK_FSPLIT) on small corpora; the default shape on a corpus
above the cut threshold (kFinMinRows)."""
import numpy as np
import pytest

import oracle as orc_mod
from test_gpu_parity import assert_same, walk_sorted

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def g():
    import __graft_entry__

    __graft_entry__.build()
    import gocask_amd

    assert gocask_amd.device_count() > 0, "no GPU visible"
    return gocask_amd


def _device_run(g, files, reset, **kw):
    # the second run of a context is the device path (the first sizes it)
    with g.ReplayContext(**kw) as ctx:
        ctx.load(files, reset)
        ctx.run()
        ctx.run()
        got, gst = ctx.fetch()
        st = ctx.stats()
    return got, gst, st


SPLITS = ["500,500", "400,300,200,100", "900,50,30,20", "10,10,10,970", "125,125,125,125,125,125,125,125"]


@pytest.mark.parametrize("split", SPLITS)
@pytest.mark.parametrize("seed", [301, 302])
def test_pieces_equal_oracle(g, orc, monkeypatch, split, seed):
    files, names = orc.gen_corpus(seed=seed, val_fixed=0, key_min=8, key_max=24, key_universe=5000,
                                  tomb_permille=20, flip_permille=20, max_file_size=3 << 20, n_files=6)
    wf, reset = walk_sorted(files, names)
    want, wst = orc.replay(wf, reset)
    monkeypatch.setenv("GCK_FSPLIT", split)
    got, gst, st = _device_run(g, wf, reset)
    assert st["device_path"] and st["n_reruns"] == 0
    assert st["ms_phase"]["finalize_side"] > 0, st["ms_phase"]  # the pieces ran
    assert_same(got, gst, want, wst)
    assert st["n_crc_fail"] == int(np.count_nonzero(want["crc_calc"] != want["crc"]))


def test_pieces_off_equals_pieces_on(g, orc, monkeypatch):
    files, names = orc.gen_corpus(seed=303, val_fixed=0, key_min=8, key_max=24, key_universe=5000,
                                  tomb_permille=20, flip_permille=20, max_file_size=3 << 20, n_files=4)
    wf, reset = walk_sorted(files, names)
    monkeypatch.setenv("GCK_FSPLIT", "0")
    a, ast, sa = _device_run(g, wf, reset)
    assert sa["ms_phase"]["finalize_side"] == 0
    monkeypatch.setenv("GCK_FSPLIT", "300,300,400")
    b, bst, sb = _device_run(g, wf, reset)
    assert sb["ms_phase"]["finalize_side"] > 0
    assert_same(b, bst, a, ast)


def test_pieces_startup_error_and_big_records(g, orc, monkeypatch):
    # 40 KiB values span several rows and piece cuts; a torn record in the
    # third file is a startup error: later records are not in the run's range
    big = b"".join(orc_mod.entry(i, b"big%05d" % i, bytes([i & 255]) * (40000 + 37 * i)) for i in range(60))
    small = b"".join(orc_mod.entry(i, b"k%06d" % i, b"v" * (i % 200)) for i in range(20000))
    torn = orc_mod.entry(7, b"torn", b"x" * 100)[:10]  # a torn header: ErrUnexpectedEOF
    files = [big, small, small + torn, big]
    reset = [True, True, True, False]
    want, wst = orc.replay(files, reset)
    assert wst["status"] != 0
    for split in ("250,250,250,250", "600,400"):
        monkeypatch.setenv("GCK_FSPLIT", split)
        got, gst, st = _device_run(g, files, reset, chunk_bytes=65536)
        assert st["ms_phase"]["finalize_side"] > 0
        assert_same(got, gst, want, wst)


def test_default_shape_above_threshold(g, monkeypatch):
    # 16 x 96 MiB (1.5 GiB >= kFinMinRows rows): the default cut; the tuples
    # equal those of the uncut pass
    kw = dict(seed=3, val_fixed=0, key_min=8, key_max=24, key_universe=300000, tomb_permille=10,
              flip_permille=10, max_file_size=96 << 20, n_files=16)
    monkeypatch.delenv("GCK_FSPLIT", raising=False)
    with g.ReplayContext() as ctx:
        ctx.encode(**kw)
        ctx.run()
        ctx.run()
        a, ast = ctx.fetch()
        st = ctx.stats()
        assert st["device_path"] and st["ms_phase"]["finalize_side"] > 0, st["ms_phase"]
        monkeypatch.setenv("GCK_FSPLIT", "0")
        ctx.run()
        b, bst = ctx.fetch()
        assert ctx.stats()["ms_phase"]["finalize_side"] == 0
    assert_same(a, ast, b, bst)
    assert ast["n_crc_fail"] > 0
