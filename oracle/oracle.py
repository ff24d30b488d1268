"""TEST INFRASTRUCTURE ONLY — ctypes wrapper over the C oracle plus a tiny
pure-Python restatement used as a second opinion on small inputs.

The oracle is the checker for the product path.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg import
this module; the product package ``gocask_amd`` never does.

Reference anchors: core/db.go:110-178 (replay), core/keydir.go:22-53 (keydir),
core/header.go:9-62 (record header), internal/crc/crc.go:5-10 (CRC-32/IEEE).
"""
from __future__ import annotations

import ctypes
import os
import struct
import subprocess
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "liboracle.so")

REC_DTYPE = np.dtype(
    [
        ("rec_off", "<u8"),
        ("file", "<u4"),
        ("key_len", "<u4"),
        ("value_pos", "<u4"),
        ("value_size", "<u4"),
        ("crc", "<u4"),
        ("ts", "<u4"),
        ("flags", "<u4"),
        ("crc_calc", "<u4"),
    ]
)
F_TOMBSTONE = 1
F_CRC_OK = 2
OK, EUNEXPECTED_EOF = 0, 1


class OrcFile(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p), ("len", ctypes.c_uint64), ("reset_after", ctypes.c_uint8)]


class OrcStatus(ctypes.Structure):
    _fields_ = [
        ("status", ctypes.c_int32),
        ("err_file", ctypes.c_uint32),
        ("err_off", ctypes.c_uint64),
        ("n_recs", ctypes.c_uint64),
        ("final_last_offset", ctypes.c_uint32),
        ("files_walked", ctypes.c_uint32),
    ]


class CorpusCfg(ctypes.Structure):
    _fields_ = [
        ("seed", ctypes.c_uint64),
        ("max_file_size", ctypes.c_uint64),
        ("n_ops", ctypes.c_uint64),
        ("n_files", ctypes.c_uint32),
        ("key_min", ctypes.c_uint32),
        ("key_max", ctypes.c_uint32),
        ("key_universe", ctypes.c_uint64),
        ("val_fixed", ctypes.c_uint32),
        ("tomb_permille", ctypes.c_uint32),
        ("flip_permille", ctypes.c_uint32),
        ("ts_base", ctypes.c_uint32),
        ("key_seed", ctypes.c_uint64),
        ("key_file", ctypes.c_uint32),
        ("pad_", ctypes.c_uint32),
    ]


_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        L.orc_crc32.restype = ctypes.c_uint32
        L.orc_crc32.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
        L.orc_crc32_fast.restype = ctypes.c_uint32
        L.orc_crc32_fast.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
        L.orc_crc32_clmul.restype = ctypes.c_uint32
        L.orc_crc32_clmul.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
        L.orc_replay.restype = ctypes.c_int
        L.orc_replay.argtypes = [ctypes.POINTER(OrcFile), ctypes.c_uint32, ctypes.c_int,
                                 ctypes.c_void_p, ctypes.c_uint64, ctypes.POINTER(OrcStatus)]
        L.orc_keydir.restype = ctypes.c_uint64
        L.orc_keydir.argtypes = [ctypes.POINTER(OrcFile), ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
        L.orc_baseline.restype = ctypes.c_uint64
        L.orc_baseline.argtypes = [ctypes.POINTER(OrcFile), ctypes.c_uint32, ctypes.c_int,
                                   ctypes.POINTER(OrcStatus)]
        L.orc_gen_sizes.restype = ctypes.c_int
        L.orc_gen_sizes.argtypes = [ctypes.POINTER(CorpusCfg), ctypes.POINTER(ctypes.c_uint64),
                                    ctypes.c_void_p, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32)]
        L.orc_gen_fill.restype = ctypes.c_int
        L.orc_gen_fill.argtypes = [ctypes.POINTER(CorpusCfg), ctypes.c_void_p, ctypes.c_uint32]
        L.orc_zipf_table.restype = None
        L.orc_zipf_table.argtypes = [ctypes.c_void_p]
        _lib = L
    return _lib


def _as_u8(b) -> np.ndarray:
    if isinstance(b, np.ndarray):
        return np.ascontiguousarray(b, dtype=np.uint8)
    return np.frombuffer(bytes(b), dtype=np.uint8)


def _files_struct(files, reset_after):
    arrs = [_as_u8(f) for f in files]
    fa = (OrcFile * max(1, len(arrs)))()
    for i, a in enumerate(arrs):
        fa[i].data = a.ctypes.data if a.size else 0
        fa[i].len = a.size
        fa[i].reset_after = 1 if reset_after[i] else 0
    return fa, arrs


def crc32(b) -> int:
    a = _as_u8(b)
    return lib().orc_crc32(a.ctypes.data if a.size else 0, a.size)


def replay(files, reset_after=None, verify_crc=True):
    """Replay files (walk order).  Returns (records ndarray[REC_DTYPE], status dict)."""
    if reset_after is None:
        reset_after = [True] * len(files)
    fa, arrs = _files_struct(files, reset_after)
    st = OrcStatus()
    L = lib()
    L.orc_replay(fa, len(arrs), 1 if verify_crc else 0, None, 0, ctypes.byref(st))
    n = st.n_recs
    out = np.zeros(max(1, n), dtype=REC_DTYPE)
    L.orc_replay(fa, len(arrs), 1 if verify_crc else 0, out.ctypes.data, n, ctypes.byref(st))
    status = dict(status=st.status, err_file=st.err_file, err_off=st.err_off, n_recs=st.n_recs,
                  final_last_offset=st.final_last_offset, files_walked=st.files_walked)
    return out[:n], status


def keydir(files, recs, reset_after=None):
    """Live keydir as {key bytes: record row} after last-writer-wins."""
    if reset_after is None:
        reset_after = [True] * len(files)
    fa, arrs = _files_struct(files, reset_after)
    recs = np.ascontiguousarray(recs, dtype=REC_DTYPE)
    live = np.zeros(max(1, len(recs)), dtype=np.uint64)
    k = lib().orc_keydir(fa, recs.ctypes.data, len(recs), live.ctypes.data)
    out = {}
    for idx in live[:k]:
        r = recs[int(idx)]
        key = bytes(arrs[int(r["file"])][int(r["rec_off"]) + 16: int(r["rec_off"]) + 16 + int(r["key_len"])])
        out[key] = r
    return out


def baseline(files, reset_after=None, verify_crc=True, bufio=True):
    """Timed CPU baseline (orc_baseline): the replay loop with the keydir map
    inline; bufio copies every record's bytes through a 4 KiB buffer as the
    reference's bufio.Reader does; verify_crc adds the CRC verdict."""
    if reset_after is None:
        reset_after = [True] * len(files)
    fa, arrs = _files_struct(files, reset_after)
    st = OrcStatus()
    live = lib().orc_baseline(fa, len(arrs), (1 if verify_crc else 0) | (2 if bufio else 0), ctypes.byref(st))
    return live, dict(status=st.status, n_recs=st.n_recs, crc_rejects=st.err_off,
                      final_last_offset=st.final_last_offset)


def zipf_table() -> np.ndarray:
    t = np.zeros(65472, dtype=np.uint32)
    lib().orc_zipf_table(t.ctypes.data)
    return t


def corpus_cfg(**kw) -> CorpusCfg:
    c = CorpusCfg()
    defaults = dict(seed=1, max_file_size=64 << 20, n_ops=0, n_files=1, key_min=16, key_max=16,
                    key_universe=0, val_fixed=1024, tomb_permille=0, flip_permille=0,
                    ts_base=1700000000, key_seed=0, key_file=0)
    defaults.update(kw)
    for k, v in defaults.items():
        setattr(c, k, v)
    return c


def gen_corpus(**kw):
    """Generate the synthetic corpus on the CPU.  Returns (files in creation
    order as numpy uint8 arrays, names)."""
    c = corpus_cfg(**kw)
    L = lib()
    n_ops = ctypes.c_uint64()
    nf = ctypes.c_uint32()
    cap = 1 << 16
    sizes = np.zeros(cap, dtype=np.uint64)
    rc = L.orc_gen_sizes(ctypes.byref(c), ctypes.byref(n_ops), sizes.ctypes.data, cap, ctypes.byref(nf))
    if rc != 0:
        raise ValueError(f"orc_gen_sizes failed: {rc}")
    files = [np.zeros(int(sizes[i]), dtype=np.uint8) for i in range(nf.value)]
    ptrs = (ctypes.c_void_p * nf.value)(*[f.ctypes.data for f in files])
    rc = L.orc_gen_fill(ctypes.byref(c), ptrs, nf.value)
    if rc != 0:
        raise ValueError(f"orc_gen_fill failed: {rc}")
    names = [f"data_{n}_{c.ts_base + n}" for n in range(nf.value)]
    return files, names


# ---------------------------------------------------------------------------
# Pure-Python second opinion (small inputs only).  Same restatement as the C
# code, written independently; uses zlib.crc32 (CRC-32/ISO-HDLC == Go IEEE).
# ---------------------------------------------------------------------------
def replay_py(files, reset_after=None):
    if reset_after is None:
        reset_after = [True] * len(files)
    last = 0
    recs = []
    status = dict(status=OK, err_file=0, err_off=0)
    for f, d in enumerate(files):
        d = bytes(d)
        p = 0
        n = len(d)
        err = False
        while True:
            if n - p == 0:
                break
            if n - p < 16:
                status = dict(status=EUNEXPECTED_EOF, err_file=f, err_off=p)
                err = True
                break
            rec = p
            hcrc, ts, ks, vs = struct.unpack_from("<IIII", d, p)
            p += 16
            tomb = ks == 0
            klen = vs if tomb else ks
            if klen > 0 and n - p == 0:
                break
            if n - p < klen:
                status = dict(status=EUNEXPECTED_EOF, err_file=f, err_off=rec)
                err = True
                break
            key = d[p:p + klen]
            p += klen
            if not tomb:
                if n - p < vs:
                    break
                p += vs
            val = d[p - vs:p]
            calc = zlib.crc32(val)
            recs.append(dict(rec_off=rec, file=f, key=key, key_len=klen,
                             value_pos=(last + 16 + ks) & 0xFFFFFFFF, value_size=vs, crc=hcrc,
                             ts=ts, tomb=tomb, crc_calc=calc, crc_ok=calc == hcrc))
            last = (last + 16 + klen) & 0xFFFFFFFF if tomb else (last + 16 + ks + vs) & 0xFFFFFFFF
        if err:
            break
        if reset_after[f]:
            last = 0
    kd = {}
    for r in recs:
        if r["tomb"]:
            kd.pop(r["key"], None)
        else:
            kd[r["key"]] = r
    return recs, kd, status, last


def entry(now: int, key: bytes, val: bytes) -> bytes:
    """core/testutil/utils.go:10-19 — canonical record encoder."""
    return struct.pack("<IIII", zlib.crc32(val), now & 0xFFFFFFFF, len(key), len(val)) + key + val


def tombstone(now: int, key: bytes) -> bytes:
    """core/db.go:245-247 — Delete writes header{CRC(key), t, 0, len(key)} || key."""
    return struct.pack("<IIII", zlib.crc32(key), now & 0xFFFFFFFF, 0, len(key)) + key


HINT_MAGIC, HINT_VERSION, HINT_BLOCK = 0x484B4347, 3, 16
_M64 = (1 << 64) - 1


def _mix64(x):
    """splitmix64's finaliser on Python ints (gocask_amd/csrc/gck_internal.h mix64d)."""
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & _M64
    return x ^ (x >> 31)


def hint_entry_check(ts, key, value_size, value_pos, crc):
    """The integrity word of one hint entry (gck_internal.h hint_entry_check,
    restated): its header words and its key's 4-byte little-endian words (the
    last one zero past the key) folded by h = (h ^ w) * K + i mod 2^64, then
    splitmix64's finaliser.  Each index entry holds the XOR of its block's
    words."""
    K = 0x9E3779B97F4A7C15
    ks = len(key)
    h = 0x2545F4914F6CDD1D ^ (ks << 32)
    for i, w in enumerate((ts, value_size, value_pos, crc)):
        h = ((h ^ w) * K + i + 1) & _M64
    padded = key + bytes(-ks % 4)
    for i in range(0, ks, 4):
        h = ((h ^ int.from_bytes(padded[i:i + 4], "little")) * K + 5 + i // 4) & _M64
    return _mix64(h)


def hint_file(entries, data_bytes):
    """One hint file (format invented here, parity unpinned: the reference has
    no hint files).  entries: [(ts, key, value_size, value_pos, crc, rec_off)]
    of one merged data file in record order; little-endian
      entries [Timestamp u32][KeySize u32][ValueSize u32][ValuePos u32][CRC u32] + key
      index   per block of HINT_BLOCK entries: [hint offset u64][data-file offset u64]
              of the block's first entry, [check u64] = the XOR of
              hint_entry_check over the block's entries
      tail    [entries u64][entry bytes u64][data-file bytes u64][magic u32][version u32]
    so a reader finds every block of entries without walking the file, and a
    record's offset in its data file (rec_off) past 4 GiB, where ValuePos wraps."""
    body, index = bytearray(), bytearray()
    for j0 in range(0, len(entries), HINT_BLOCK):
        blk = entries[j0:j0 + HINT_BLOCK]
        check = 0
        for ts, key, vs, vpos, crc, _ in blk:
            check ^= hint_entry_check(ts, key, vs, vpos, crc)
        index += struct.pack("<QQQ", len(body), blk[0][5], check)
        for ts, key, vs, vpos, crc, _ in blk:
            body += struct.pack("<IIIII", ts, len(key), vs, vpos, crc) + key
    tail = struct.pack("<QQQII", len(entries), len(body), data_bytes, HINT_MAGIC, HINT_VERSION)
    return bytes(body + index + tail)


def compact(files, recs, reset_after, max_file_size):
    """Merge (compaction) restated — the reference's roadmap item "merging and
    hint files" (README.md:60), defined as: the live records of the keydir
    (orc_keydir: last writer wins, Puts only, core/keydir.go:22-49) in walk
    order, Put into a fresh database with MaxDataFileSize = max_file_size —
    DB.Put (core/db.go:185-212) rotates when the active file's size + the
    entry > MaxDataFileSize (rotateDataFile, :214-231; the fresh database's
    first file starts empty) — each record's bytes verbatim.  Per merged file
    a hint file (hint_file): per record [Timestamp][KeySize][ValueSize]
    [ValuePos][CRC] + key, ValuePos = the value's offset in the merged file
    mod 2^32 as core/keydir.go:25 sets it, CRC = the header's (kdEntry.CRC),
    so the keydir can be filled without reading the data files.
    Returns (list of data-file bytes, list of hint-file bytes)."""
    kd = keydir(files, recs, reset_after)
    live = sorted(kd.values(), key=lambda r: (int(r["file"]), int(r["rec_off"])))
    data, ents = [bytearray()], [[]]
    for r in live:
        f, o = files[int(r["file"])], int(r["rec_off"])
        kl, vs = int(r["key_len"]), int(r["value_size"])
        b = bytes(f[o:o + 16 + kl + vs])
        if len(data[-1]) + len(b) > max_file_size:
            data.append(bytearray())
            ents.append([])
        vpos = (len(data[-1]) + 16 + kl) & 0xFFFFFFFF
        ents[-1].append((int(r["ts"]), b[16:16 + kl], vs, vpos, int(r["crc"]), len(data[-1])))
        data[-1] += b
    return [bytes(d) for d in data], [hint_file(e, len(d)) for e, d in zip(ents, data)]


def parse_hints(h):
    """Hint entries of one hint file (hint_file's format), walked from the
    start and checked against its index and tail: [(timestamp, key,
    value_size, value_pos, crc, rec_off)]."""
    n, nbytes, dbytes, magic, ver = struct.unpack_from("<QQQII", h, len(h) - 32)
    nb = (n + HINT_BLOCK - 1) // HINT_BLOCK
    assert magic == HINT_MAGIC and ver == HINT_VERSION and len(h) == nbytes + 24 * nb + 32
    out, p, d = [], 0, 0
    for j in range(n):
        if j % HINT_BLOCK == 0:
            assert struct.unpack_from("<QQ", h, nbytes + 24 * (j // HINT_BLOCK)) == (p, d)
        ts, kl, vs, vpos, crc = struct.unpack_from("<IIIII", h, p)
        out.append((ts, bytes(h[p + 20:p + 20 + kl]), vs, vpos, crc, d))
        p += 20 + kl
        d += 16 + kl + vs
    assert p == nbytes and d == dbytes
    for b in range(nb):
        x = 0
        for ts, key, vs, vpos, crc, _ in out[b * HINT_BLOCK:(b + 1) * HINT_BLOCK]:
            x ^= hint_entry_check(ts, key, vs, vpos, crc)
        assert struct.unpack_from("<Q", h, nbytes + 24 * b + 16)[0] == x
    return out