"""GCK_OPT_FUSED (experimental): boundary discovery fused into the streaming
CRC pass must give the records, verdicts, status and final lastOffset of the
standard path, i.e. the oracle's, bit for bit.  The fused path runs from a
context's second run on (the first sizes the record table on the host path);
stats()["n_reruns"] counts runs it handed back to the standard path."""
import numpy as np
import pytest

from golden_cases import case_names, load_case
from test_gpu_parity import CORPORA, assert_same, walk_sorted

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def g():
    import __graft_entry__

    __graft_entry__.build()
    import gocask_amd

    assert gocask_amd.device_count() > 0, "no GPU visible"
    return gocask_amd


def _fused_twice(g, files, reset, **kw):
    with g.ReplayContext(flags=g.core.OPT_FUSED, **kw) as ctx:
        ctx.load(files, reset)
        ctx.run()
        ctx.run()
        got, st = ctx.fetch()
        stats = ctx.stats()
    return got, st, stats


@pytest.mark.parametrize("name", case_names())
def test_fused_golden(g, orc, name):
    meta, files, reset = load_case(name)
    want, wst = orc.replay(files, reset)
    got, gst, stats = _fused_twice(g, files, reset)
    assert_same(got, gst, want, wst)


@pytest.mark.parametrize("chunk", [4096, 1 << 15, 1 << 19])
@pytest.mark.parametrize("ci", range(len(CORPORA)))
def test_fused_random(g, orc, ci, chunk):
    files, names = orc.gen_corpus(**CORPORA[ci])
    wf, reset = walk_sorted(files, names)
    want, wst = orc.replay(wf, reset)
    got, gst, stats = _fused_twice(g, wf, reset, chunk_bytes=chunk)
    assert_same(got, gst, want, wst)
    # the fused path hands a run back only when a chunk holds more records than
    # its stage (1024) or an 8 KiB step more than 64
    per_chunk = np.unique(want["file"].astype(np.uint64) << np.uint64(40) | want["rec_off"] // np.uint64(chunk),
                          return_counts=True)[1]
    per_step = np.unique(want["file"].astype(np.uint64) << np.uint64(40) | want["rec_off"] // np.uint64(8192),
                         return_counts=True)[1]
    if per_chunk.max() <= 1024 and per_step.max() <= 64 and chunk >= 1 << 15:
        assert stats["device_path"] and stats["n_reruns"] == 0, stats
    if per_chunk.max() > 1024:
        assert not stats["device_path"], stats


def test_fused_c3_shape(g):
    # C3 shape at 1/8 scale, device-encoded: fused and standard runs agree
    kw = dict(seed=3, val_fixed=0, key_min=8, key_max=24, key_universe=600000, tomb_permille=10,
              flip_permille=10, max_file_size=256 << 20, n_files=16)
    with g.ReplayContext() as ctx:
        ctx.encode(**kw)
        ctx.run()
        ctx.run()
        want, wst = ctx.fetch()
    with g.ReplayContext(flags=g.core.OPT_FUSED) as ctx:
        ctx.encode(**kw)
        ctx.run()
        ctx.run()
        got, gst = ctx.fetch()
        stats = ctx.stats()
    assert stats["device_path"] and stats["n_reruns"] == 0, stats
    assert_same(got, gst, want, wst)


def test_fused_values_that_look_like_records(g, orc):
    # speculation lands inside values: validation rounds stream chunks again
    import oracle as orc_mod

    rng = np.random.default_rng(9)
    parts = []
    for i in range(400):
        inner = b"".join(orc_mod.entry(j, b"inner%d" % j, bytes(rng.integers(0, 256, 300, dtype=np.uint8)))
                         for j in range(int(rng.integers(1, 30))))
        parts.append(orc_mod.entry(i, b"outer%05d" % i, inner))
    data = b"".join(parts)
    want, wst = orc.replay([data], [True])
    for chunk in (4096, 1 << 14):
        got, gst, stats = _fused_twice(g, [data], [True], chunk_bytes=chunk)
        assert_same(got, gst, want, wst)
