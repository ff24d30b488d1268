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


def _raw_encode(keys_t, koff, vals_t, voff, ts, tomb, out, out_off):
    import ctypes

    from gocask_amd import _lib

    total = ctypes.c_uint64(0)
    return _lib.load().gck_encode_batch(keys_t.data_ptr(), koff.data_ptr(), vals_t.data_ptr(), voff.data_ptr(),
                                        ts.data_ptr(), tomb.data_ptr(), len(ts), out.data_ptr(), out.numel(),
                                        out_off.data_ptr(), ctypes.byref(total), None), total.value


def test_encode_batch_exact_size_and_alignment():
    """Exact-size blobs (no padding) encode correctly; blobs that do not start
    on a 4-byte boundary are refused (the kernel reads dwords)."""
    import torch

    from gocask_amd import _lib

    ops = [(11, b"abc", b"12345"), (12, b"k" * 37, bytes(range(200)) * 3), (13, b"z", None), (14, b"tail", b"x" * 4097)]
    keys = b"".join(k for _, k, _ in ops)
    vals = b"".join(v for _, _, v in ops if v is not None)
    koff = np.cumsum([0] + [len(k) for _, k, _ in ops]).astype(np.int64)
    voff = np.cumsum([0] + [0 if v is None else len(v) for _, _, v in ops]).astype(np.int64)

    def dev(b, extra_front=0):
        t = torch.empty(len(b) + extra_front, dtype=torch.uint8, device="cuda")
        t[extra_front:] = torch.frombuffer(bytearray(b), dtype=torch.uint8).cuda()
        return t[extra_front:]

    d_koff, d_voff = torch.from_numpy(koff).cuda(), torch.from_numpy(voff).cuda()
    ts = torch.tensor([t for t, _, _ in ops], dtype=torch.int32, device="cuda")
    tomb = torch.tensor([v is None for _, _, v in ops], dtype=torch.uint8, device="cuda")
    need = sum(16 + len(k) + (0 if v is None else len(v)) for _, k, v in ops)
    out = torch.zeros(need, dtype=torch.uint8, device="cuda")
    out_off = torch.zeros(len(ops) + 1, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    rc, total = _raw_encode(dev(keys), d_koff, dev(vals), d_voff, ts, tomb, out, out_off)
    assert rc == _lib.GCK_OK and total == need
    assert bytes(out.cpu().numpy()) == _expected(ops)
    # too small an output: refused, the size needed reported, nothing written
    small = torch.zeros(need - 1, dtype=torch.uint8, device="cuda")
    rc, total = _raw_encode(dev(keys), d_koff, dev(vals), d_voff, ts, tomb, small, out_off)
    assert rc == _lib.GCK_EINVAL and total == need
    assert int(small.sum()) == 0
    rc, _ = _raw_encode(dev(keys, 1), d_koff, dev(vals), d_voff, ts, tomb, out, out_off)
    assert rc == _lib.GCK_EINVAL
    rc, _ = _raw_encode(dev(keys), d_koff, dev(vals, 3), d_voff, ts, tomb, out, out_off)
    assert rc == _lib.GCK_EINVAL


@pytest.mark.parametrize("seed", [21, 22, 23])
def test_encode_batch_piece_edges(seed):
    """Key and value lengths around the 16 B pieces and 1 KiB rows of the
    copy (a region shorter than a piece, exactly one or two pieces, one byte
    over), tombstones with long keys, and the batch's first records, whose
    short keys and values are copied byte by byte (no 16 B before them in the
    blob)."""
    from gocask_amd import core

    rng = random.Random(seed)
    klens = [1, 2, 15, 16, 17, 31, 32, 33, 48, 100]
    vlens = [0, 1, 2, 15, 16, 17, 31, 32, 33, 1007, 1008, 1023, 1024, 1025, 2048]
    ops = [(1, b"a", b"b"), (2, b"cd", b""), (3, b"e" * 15, b"f" * 3)]
    for i in range(3000):
        k = rng.randbytes(rng.choice(klens))
        if rng.random() < 0.1:
            ops.append((100 + i, k, None))
        else:
            ops.append((100 + i, k, rng.randbytes(rng.choice(vlens + [rng.randint(0, 5000)]))))
    out, off = core.encode_batch(ops)
    assert bytes(out.cpu().numpy()) == _expected(ops)


@pytest.mark.parametrize("seed", [31, 32])
def test_encode_batch_random_large(seed):
    """100 K records of every size class at once -- many per 16 B piece, per
    1 KiB stripe and per 64 KiB unit, values past a unit -- so the wave path's
    stripe stores, the lane path's pieces and the per-record pieces of
    neighbouring records (often in one wavefront, sometimes in two) all meet;
    byte-exact against the oracle's serializeEntry."""
    from gocask_amd import core

    rng = np.random.default_rng(seed)
    n = 100_000
    kl = rng.integers(1, 65, n)
    cls = rng.random(n)
    vl = np.where(cls < 0.6, rng.integers(0, 300, n),
                  np.where(cls < 0.95, rng.integers(300, 4096, n), rng.integers(4096, 70_000, n)))
    tomb = rng.random(n) < 0.05
    blob = rng.integers(0, 256, int(kl.sum() + vl.sum()), dtype=np.uint8).tobytes()
    ops, o = [], 0
    for i in range(n):
        k = blob[o:o + int(kl[i])]
        o += int(kl[i])
        v = None if tomb[i] else blob[o:o + int(vl[i])]
        o += int(vl[i])
        ops.append((int(rng.integers(0, 2**32)), k, v))
    out, off = core.encode_batch(ops)
    exp = _expected(ops)
    got = bytes(out.cpu().numpy())
    assert len(got) == len(exp)
    if got != exp:
        a = np.frombuffer(got, np.uint8) != np.frombuffer(exp, np.uint8)
        raise AssertionError(f"first differing byte {int(np.argmax(a))} of {len(exp)}")
