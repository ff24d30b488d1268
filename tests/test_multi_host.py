"""gck_replay_multi's host-side orchestration on the CPU (libgocask_diag.so's
entries over the library's own code, no GPU): the global outcome over several
shards and the exchange's receive layout.

The rule: the first startup error in walk order ends the whole walk
(/root/reference/core/db.go:134-138, /root/reference/internal/fs/disk.go:134-141):
its shard's records before the error count, later shards contribute nothing;
lastOffset after the walk is the last contributing shard's (cuts follow files
that reset it, /root/reference/core/db.go:117-119).  gocask_amd/shard.py's
resolve_status is the Python statement of the same rule; both must agree."""
import random

import numpy as np
import pytest

EOF = 1


def _outcome(nfiles, status=0, err_file=0, err_off=0, walked=None, last=0, rej=0):
    return dict(status=status, nfiles=nfiles, err_file=err_file, err_off=err_off,
                files_walked=nfiles if walked is None else walked, final_last_offset=last, n_crc_fail=rej)


@pytest.fixture(scope="module")
def g():
    import gocask_amd

    return gocask_amd


def test_resolve_no_error(g):
    sh = [_outcome(3, last=0, rej=2), _outcome(0), _outcome(4, last=77, rej=5)]
    st, contrib = g.multi_resolve(sh, 7)
    assert st["status"] == 0 and st["files_walked"] == 7 and st["final_last_offset"] == 77
    assert st["n_crc_fail"] == 7 and contrib == [True, True, True]


def test_resolve_error_in_middle_shard(g):
    sh = [_outcome(3, rej=1), _outcome(4, status=EOF, err_file=2, err_off=123, walked=3, last=55, rej=4),
          _outcome(5, last=9, rej=100), _outcome(2, status=EOF, err_file=0, err_off=1, walked=1)]
    st, contrib = g.multi_resolve(sh, 14)
    assert st["status"] == EOF
    assert (st["err_file"], st["err_off"], st["files_walked"]) == (3 + 2, 123, 3 + 3)
    assert st["final_last_offset"] == 55 and st["n_crc_fail"] == 5
    assert contrib == [True, True, False, False]


def test_resolve_error_in_first_and_empty_shards(g):
    sh = [_outcome(0), _outcome(2, status=EOF, err_file=0, err_off=16, walked=1, last=3), _outcome(0)]
    st, contrib = g.multi_resolve(sh, 2)
    assert (st["status"], st["err_file"], st["err_off"], st["files_walked"]) == (EOF, 0, 16, 1)
    assert contrib == [True, True, False]
    # an empty shard's status is ignored (it walks no file)
    st, contrib = g.multi_resolve([_outcome(0, status=EOF), _outcome(1, last=4)], 1)
    assert st["status"] == 0 and st["final_last_offset"] == 4 and contrib == [True, True]


def test_resolve_matches_shard_py_random(g):
    """Random outcomes: the library's rule equals shard.resolve_status."""
    from gocask_amd import shard

    rng = random.Random(7)
    for _ in range(300):
        n = rng.randint(1, 8)
        sh = []
        for _s in range(n):
            nf = rng.choice([0, 1, 2, 5])
            if nf and rng.random() < 0.25:
                ef = rng.randrange(nf)
                sh.append(_outcome(nf, EOF, ef, rng.randrange(1 << 40), ef + 1, rng.randrange(1 << 32),
                                   rng.randrange(50)))
            else:
                sh.append(_outcome(nf, last=rng.randrange(1 << 32), rej=rng.randrange(50)))
        nfiles = sum(o["nfiles"] for o in sh)
        st, contrib = g.multi_resolve(sh, nfiles)
        per_rank = [dict(status=o["status"] if o["nfiles"] else 0, err_file=o["err_file"], err_off=o["err_off"],
                         files_walked=o["files_walked"], final_last_offset=o["final_last_offset"],
                         n_files=o["nfiles"]) for o in sh]
        want, wc = shard.resolve_status(per_rank)
        assert contrib == wc
        for k in ("status", "final_last_offset"):
            assert st[k] == want[k], (k, sh, st, want)
        if want["status"]:
            assert (st["err_file"], st["err_off"], st["files_walked"]) == (
                want["err_file"], want["err_off"], want["files_walked"])
        assert st["n_crc_fail"] == sum(o["n_crc_fail"] for o, c in zip(sh, contrib) if c and o["nfiles"])


def test_recv_offsets(g):
    rng = np.random.default_rng(3)
    for nsrc, nown in ((1, 1), (3, 2), (7, 4), (40, 8), (0, 3)):
        c = rng.integers(0, 1000, size=(nsrc, nown), dtype=np.uint64)
        off = g.multi_recv_offsets(c)
        assert off.shape == (nown, nsrc + 1)
        for p in range(nown):
            want = np.concatenate([[0], np.cumsum(c[:, p])]).astype(np.uint64)
            assert np.array_equal(off[p], want)
