"""Bulk serializeEntry on the device (row f4, gck_encode_batch) against the
oracle's canonical encoders (oracle.entry = core/testutil/utils.go:10-19,
oracle.tombstone = core/db.go:245-247), and a replay round trip of the bytes
it writes."""
import random

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu


def _expected(ops):
    return b"".join(oracle.entry(t, k, v) if v is not None else oracle.tombstone(t, k) for t, k, v in ops)


def _ops(seed, n, vmax):
    rng = random.Random(seed)
    ops = []
    for i in range(n):
        k = rng.randbytes(rng.randint(1, 40))
        if rng.random() < 0.1:
            ops.append((1_700_000_000 + i, k, None))
        else:
            ops.append((1_700_000_000 + i, k, rng.randbytes(rng.choice([0, 1, 7, 63, 64, 65, rng.randint(0, vmax)]))))
    return ops


@pytest.mark.parametrize("seed,n,vmax", [(1, 1, 100), (2, 300, 300), (3, 2000, 5000), (4, 40, 200_000)])
def test_encode_batch_matches_oracle(seed, n, vmax):
    from gocask_amd import core

    ops = _ops(seed, n, vmax)
    out, off = core.encode_batch(ops)
    exp = _expected(ops)
    assert bytes(out.cpu().numpy()) == exp
    sizes = [16 + len(k) + (0 if v is None else len(v)) for _, k, v in ops]
    assert off.cpu().numpy().tolist() == [0] + np.cumsum(sizes).tolist()


def test_encode_batch_empty_and_zero_length():
    from gocask_amd import core

    out, off = core.encode_batch([])
    assert out.numel() == 0 and off.cpu().numpy().tolist() == [0]
    ops = [(5, b"k", b""), (7, b"gone", None), (2**32 + 9, b"x" * 64, b"y" * 4096),
           (8, bytes(range(256)) * 20, None), (9, b"q" * 3000, bytes(range(7)) * 300), (10, b"z", b"")]
    out, _ = core.encode_batch(ops)
    assert bytes(out.cpu().numpy()) == _expected(ops)


@pytest.mark.parametrize("bad", [(6, b"", b"v"), (6, b"", b""), (6, b"", None)])
def test_encode_batch_rejects_empty_key(bad):
    # DB.Put and DB.Delete reject an empty key with ErrInvalidKey
    # (core/db.go:186-188; Delete through get, :238-241, :294-297)
    from gocask_amd import _lib, core

    with pytest.raises(_lib.GckError) as e:
        core.encode_batch([(1, b"a", b"b"), bad])
    assert e.value.code == _lib.GCK_EINVALID_KEY


def test_encode_batch_replays():
    """The encoded file replays (device path) to the oracle's records and keydir."""
    from gocask_amd import core

    ops = _ops(9, 500, 3000)
    out, _ = core.encode_batch(ops)
    data = bytes(out.cpu().numpy())
    arr = np.frombuffer(data, dtype=np.uint8).copy()
    recs, st = core.replay([arr])
    orecs, ost = oracle.replay([arr])
    assert st["status"] == ost["status"] == 0
    assert len(recs) == len(orecs) == len(ops)
    assert (recs == orecs).all()
    assert st["n_crc_fail"] == 0
