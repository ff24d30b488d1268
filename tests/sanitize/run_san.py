"""TEST INFRASTRUCTURE ONLY.  Runs under LD_PRELOAD=libasan (tests/test_sanitize.py):
the sanitizer builds of the oracle and of the host mirror db.cpp replay every
golden fixture, random corpora, and the Open/Get/Keys disk cases the
reference's tests use (internal/fs/disk_test.go:64-88, db_test.go:16-74,
core/db_test.go:494-500).  Any ASan/UBSan report aborts the process."""
import ctypes
import os
import sys
import tempfile
import zlib

HERE = os.path.dirname(os.path.abspath(__file__))
TESTS = os.path.dirname(HERE)
ROOT = os.path.dirname(TESTS)
sys.path[:0] = [TESTS, os.path.join(ROOT, "oracle")]

import numpy as np  # noqa: E402

import oracle  # noqa: E402
from golden_cases import case_names, check_case, load_case  # noqa: E402

assert "libasan" in open("/proc/self/maps").read(), "run under LD_PRELOAD=libasan (tests/test_sanitize.py)"
oracle.LIB_PATH = os.path.join(HERE, "build", "liboracle_san.so")
oracle._lib = None

# ---- the oracle under the sanitizers: every fixture and random corpora ----
for name in case_names():
    meta, files, reset = load_case(name)
    recs, st = oracle.replay(files, reset)
    check_case(meta, files, recs, oracle.keydir(files, recs, reset), st)
    oracle.baseline(files, reset)
    oracle.baseline(files, reset, verify_crc=False)
for seed in (1, 2, 3):
    files, names = oracle.gen_corpus(seed=seed, val_fixed=0, key_min=8, key_max=30, key_universe=200,
                                     tomb_permille=100, flip_permille=50, max_file_size=1 << 18, n_files=4)
    recs, st = oracle.replay(files)
    oracle.keydir(files, recs)
    for cut in (1, 7, 16, 17, 40):  # truncated tails: every EOF class
        t = [f[:max(0, len(f) - cut)] for f in files]
        oracle.replay(t)
print("oracle ok")

# ---- the host mirror (db.cpp) ----
H = ctypes.CDLL(os.path.join(HERE, "build", "libgck_host_san.so"))
vp, P = ctypes.c_void_p, ctypes.POINTER


class Cfg(ctypes.Structure):
    _fields_ = [("max_data_file_size", ctypes.c_int64), ("data_dir", ctypes.c_char_p)]


H.gck_db_open.argtypes = [ctypes.c_char_p, P(Cfg), vp, P(vp), ctypes.c_char_p, ctypes.c_size_t]
H.gck_db_open_mem.argtypes = [vp, ctypes.c_uint64, vp, P(vp), ctypes.c_char_p, ctypes.c_size_t]
H.gck_db_get.argtypes = [vp, ctypes.c_char_p, ctypes.c_uint32, P(vp), P(ctypes.c_uint64)]
H.gck_db_keys.argtypes = [vp]
H.gck_db_keys.restype = ctypes.c_uint64
H.gck_db_key.argtypes = [vp, ctypes.c_uint64, P(vp), P(ctypes.c_uint32)]
H.gck_db_active_file.argtypes = [vp]
H.gck_db_active_file.restype = ctypes.c_char_p
H.gck_db_nfiles.argtypes = [vp]
H.gck_db_nfiles.restype = ctypes.c_uint32
H.gck_db_file_name.argtypes = [vp, ctypes.c_uint32]
H.gck_db_file_name.restype = ctypes.c_char_p
H.gck_db_last_offset.argtypes = [vp]
H.gck_db_last_offset.restype = ctypes.c_uint32
H.gck_db_close.argtypes = [vp]


def open_disk(data_dir, name):
    h, err = vp(), ctypes.create_string_buffer(256)
    c = Cfg(1 << 30, data_dir.encode())
    rc = H.gck_db_open(name.encode(), ctypes.byref(c), None, ctypes.byref(h), err, 256)
    return rc, h, err.value.decode()


def keys(h):
    out = []
    k, kl = vp(), ctypes.c_uint32()
    for i in range(H.gck_db_keys(h)):
        assert H.gck_db_key(h, i, ctypes.byref(k), ctypes.byref(kl)) == 0
        out.append(ctypes.string_at(k, kl.value))
    return sorted(out)


def get(h, key):
    v, n = vp(), ctypes.c_uint64()
    rc = H.gck_db_get(h, key, len(key), ctypes.byref(v), ctypes.byref(n))
    return rc, (ctypes.string_at(v, n.value) if rc == 0 and n.value else b"")


with tempfile.TemporaryDirectory() as tmp:
    # empty db: Disk.Open creates data_0_<unix>.csk (internal/fs/disk.go:56-67), Keys() = []
    rc, h, _ = open_disk(tmp, "fresh")
    assert rc == 0 and keys(h) == [] and H.gck_db_nfiles(h) == 1
    made = os.listdir(os.path.join(tmp, "fresh"))
    assert len(made) == 1 and made[0].startswith("data_0_") and made[0].endswith(".csk")
    assert get(h, b"")[0] == 8 and get(h, b"nope")[0] == 6  # ErrInvalidKey, ErrKeyNotFound
    H.gck_db_close(h)

    # rotated files + foo.txt + a nested directory, lexical walk order
    files, names = oracle.gen_corpus(seed=21, val_fixed=0, key_min=8, key_max=12, key_universe=500,
                                     tomb_permille=30, flip_permille=20, max_file_size=1 << 16, n_files=12)
    d = os.path.join(tmp, "mydb")
    os.makedirs(os.path.join(d, "a_sub"))  # walked first; not the active file (a directory would fail Open)
    for f, n in zip(files, names):
        open(os.path.join(d, n + ".csk"), "wb").write(f.tobytes())
    open(os.path.join(d, "foo.txt"), "wb").write(b"not a data file")
    extra = oracle.entry(7, b"nested", b"value") + oracle.tombstone(8, b"gone")
    open(os.path.join(d, "a_sub", "data_x.csk"), "wb").write(extra)
    rc, h, _ = open_disk(tmp, "mydb")
    assert rc == 0, rc
    assert H.gck_db_active_file(h) == b"foo"
    walk = sorted(names)
    got_names = [H.gck_db_file_name(h, i).decode() for i in range(H.gck_db_nfiles(h))]
    assert got_names == ["data_x"] + walk, got_names
    wf = [np.frombuffer(extra, np.uint8)] + [files[names.index(n)] for n in walk]
    recs, st = oracle.replay(wf, [True] * len(wf))
    kd = oracle.keydir(wf, recs, [True] * len(wf))
    assert keys(h) == sorted(kd)
    bad = 0
    for k, r in kd.items():
        rc, v = get(h, k)
        if int(r["flags"]) & 2:
            # Get of a nested file's key reads <path>/<Name>.csk (disk.go:147-159): absent here
            assert rc == (5 if k == b"nested" else 0), (k, rc)
            if rc == 0:
                assert zlib.crc32(v) == int(r["crc"])
        else:
            assert rc == 7, (k, rc)  # ErrCRCFailed
            bad += 1
    assert bad > 0 and H.gck_db_last_offset(h) == st["final_last_offset"]
    H.gck_db_close(h)

    # a path that is a file, not a folder
    open(os.path.join(tmp, "plain"), "wb").write(b"x")
    assert open_disk(tmp, "plain")[0] == 9

    # startup error: the DB comes back with the records before it
    meta, files, reset = load_case("partial_write_desync")
    d = os.path.join(tmp, "broken")
    os.makedirs(d)
    open(os.path.join(d, "data_0_1.csk"), "wb").write(files[0].tobytes())
    rc, h, err = open_disk(tmp, "broken")
    assert rc == 1 and err == "gocask: startup error: unexpected EOF" and keys(h) == [b"key", b"user"]
    H.gck_db_close(h)

# in-memory FS: the 1000-Put testdata file (db_test.go:39-74)
meta, files, reset = load_case("datatxt_1000_puts")
h, err = vp(), ctypes.create_string_buffer(256)
buf = files[0].tobytes()
assert H.gck_db_open_mem(buf, len(buf), None, ctypes.byref(h), err, 256) == 0
assert keys(h) == sorted(k.encode() for k in meta["expect"])
for k, e in meta["expect"].items():
    assert get(h, k.encode()) == (0, e["value"].encode())
H.gck_db_close(h)
print("host ok")
