"""Vectorised restatement of the corpus spec's hash (DESIGN.md "Corpus") for
size-independent property checks at full scale (which records carry a flipped
bit, which are tombstones) without running the oracle on 32 GiB."""
import numpy as np

_G = np.uint64(0x9E3779B97F4A7C15)
_C1 = np.uint64(0xBF58476D1CE4E5B9)
_C2 = np.uint64(0x94D049BB133111EB)
_T = 0xD6E8FEB86659FD93


def mix64(x):
    x = np.asarray(x, dtype=np.uint64) + _G
    x = (x ^ (x >> np.uint64(30))) * _C1
    x = (x ^ (x >> np.uint64(27))) * _C2
    return x ^ (x >> np.uint64(31))


def H(seed, tag, i):
    k = mix64(np.array([(seed ^ (tag * _T)) & ((1 << 64) - 1)], dtype=np.uint64))[0]
    return mix64(np.asarray(i, dtype=np.uint64) + k)


def expected_flips(seed, ops, flip_permille, tomb_permille):
    """Boolean per op index: a bit of the value was flipped after the CRC."""
    ops = np.asarray(ops, dtype=np.uint64)
    tomb = (H(seed, 3, ops) % np.uint64(1000)) < np.uint64(tomb_permille) if tomb_permille else np.zeros(len(ops), bool)
    flip = (H(seed, 4, ops) % np.uint64(1000)) < np.uint64(flip_permille)
    return flip & ~tomb
