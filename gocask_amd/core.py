"""Python mirror of the reference surface around cold-start replay.

Names, argument meaning and error behaviour follow the Go reference so tests
read like its own: ``NewDB`` (core/db.go:90-108) and ``Open`` (db.go:29-59)
return ``(db, err)``; ``DB.Get`` returns ``(value, err)`` with ``ErrKeyNotFound``
/ ``ErrCRCFailed`` / ``ErrInvalidKey`` (core/db.go:13-31); ``DB.Keys``
(core/db.go:318-324).  Everything below the ctypes calls is native: the C++
host mirror in gocask_amd/csrc/db.cpp and the HIP pipeline in replay.hip.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass

import numpy as np

from . import _lib
from ._lib import (F_CRC_OK, F_TOMBSTONE, GCK_ECRC_FAILED, GCK_EINVAL, GCK_EINVALID_KEY, GCK_EKEY_NOT_FOUND, GCK_OK,
                   GCK_EUNEXPECTED_EOF, KD_ENTRY_DTYPE, REC_DTYPE, GckCorpusCfg, GckFile, GckOpts, GckResult, GckStats, check)

InMemoryDB = "in:mem:db"  # core/db.go:32-34

KB = 1024
MB = KB * 1024
GB = MB * 1024
TB = GB * 1024


class GoCaskError(Exception):
    pass


ErrKeyNotFound = GoCaskError("gocask: key not found")
ErrPartialWrite = GoCaskError("gocask: key/value pair not fully written")
ErrCRCFailed = GoCaskError("gocask: crc check failed for db entry (value is corrupted)")
ErrInvalidKey = GoCaskError("gocask: key should not be empty or nil")
ErrInvalidValue = GoCaskError("gocask: value should not be nil")
ErrUnexpectedEOF = GoCaskError("unexpected EOF")


class StartupError(GoCaskError):
    """fmt.Errorf("gocask: startup error: %w", err) (core/db.go:138)."""

    def __init__(self, wrapped=ErrUnexpectedEOF):
        super().__init__(f"gocask: startup error: {wrapped}")
        self.wrapped = wrapped

    def is_(self, err):
        return err is self.wrapped or err is self


@dataclass
class Config:  # core.Config (core/db.go:84-87)
    MaxDataFileSize: int = 2 * GB
    DataDir: str = "./"


DefaultConfig = Config()  # core/db.go:78-81


class Disk:
    """Marker for fs.NewDisk() (internal/fs/disk.go:42-48)."""


class InMemory:
    """fs.NewInMemory(): one file "data" that is also the active file
    (internal/fs/memory.go:38-80).  ``data`` holds the bytes written so far."""

    def __init__(self, data: bytes = b""):
        self.data = bytes(data)


def NewDisk():
    return Disk()


def NewInMemory(data: bytes = b""):
    return InMemory(data)


def _opts(device=0, chunk_bytes=0, max_key=0, chunk_cap=0, spec_window=0, max_resident=0, keys=False, live=False):
    o = GckOpts()
    o.device = device
    o.chunk_bytes = chunk_bytes
    o.max_key = max_key
    o.chunk_cap = chunk_cap
    o.flags = (_lib.OPT_KEYS if keys else 0) | (_lib.OPT_LIVE if live else 0)
    o.spec_window = spec_window
    o.max_resident = max_resident
    return o


class DB:
    """core.DB restricted to the replayed state: keydir, Get, Keys, Close."""

    def __init__(self, handle):
        self._h = handle
        self._L = _lib.load()

    def Get(self, key: bytes):
        if key is None:
            key = b""
        val = ctypes.c_void_p()
        n = ctypes.c_uint64()
        rc = self._L.gck_db_get(self._h, key, len(key), ctypes.byref(val), ctypes.byref(n))
        if rc == GCK_OK:
            return ctypes.string_at(val, n.value) if n.value else b"", None
        err = {GCK_EKEY_NOT_FOUND: ErrKeyNotFound, GCK_ECRC_FAILED: ErrCRCFailed,
               GCK_EINVALID_KEY: ErrInvalidKey}.get(rc)
        if err is None:
            err = GoCaskError(f"gocask: read failed ({rc})")
        return None, err

    def Keys(self):
        n = self._L.gck_db_keys(self._h)
        out = []
        k = ctypes.c_void_p()
        kl = ctypes.c_uint32()
        for i in range(n):
            check(self._L.gck_db_key(self._h, i, ctypes.byref(k), ctypes.byref(kl)))
            out.append(ctypes.string_at(k, kl.value).decode("utf-8", "surrogateescape"))
        return out

    def Entry(self, key: bytes):
        """The kdEntry for key (core/keydir.go:3-9) or None."""
        crc, ts, pos, size = (ctypes.c_uint32() for _ in range(4))
        f = ctypes.c_char_p()
        rc = self._L.gck_db_entry(self._h, key, len(key), ctypes.byref(crc), ctypes.byref(ts), ctypes.byref(pos),
                                  ctypes.byref(size), ctypes.byref(f))
        if rc != GCK_OK:
            return None
        return dict(CRC=crc.value, Timestamp=ts.value, ValuePos=pos.value, ValueSize=size.value,
                    File=f.value.decode())

    @property
    def last_offset(self):
        return self._L.gck_db_last_offset(self._h)

    @property
    def active_file(self):
        return self._L.gck_db_active_file(self._h).decode()

    def files(self):
        return [self._L.gck_db_file_name(self._h, i).decode() for i in range(self._L.gck_db_nfiles(self._h))]

    def Close(self):
        if self._h:
            self._L.gck_db_close(self._h)
            self._h = None
        return None

    def __del__(self):
        try:
            self.Close()
        except Exception:
            pass


def NewDB(dbpath: str, fs, time=None, cfg: Config = DefaultConfig, device: int = 0):
    """core.NewDB: returns (db, err).  On a startup error the DB is still
    returned with the partially replayed keydir, as the reference does."""
    L = _lib.load()
    h = ctypes.c_void_p()
    err = ctypes.create_string_buffer(256)
    if isinstance(fs, InMemory):
        buf = np.frombuffer(fs.data, dtype=np.uint8) if fs.data else np.zeros(1, np.uint8)
        rc = L.gck_db_open_mem(buf.ctypes.data, len(fs.data), ctypes.byref(_opts(device)), ctypes.byref(h), err, 256)
    else:
        c = _lib.GckConfig()
        c.max_data_file_size = cfg.MaxDataFileSize
        c.data_dir = cfg.DataDir.encode()
        rc = L.gck_db_open(dbpath.encode(), ctypes.byref(c), ctypes.byref(_opts(device)), ctypes.byref(h), err, 256)
    if rc == GCK_OK:
        return DB(h), None
    if rc == GCK_EUNEXPECTED_EOF:
        return DB(h), StartupError()
    check(rc)


def WithMaxDataFileSize(n: int):  # db.go:63-73
    def opt(c: Config) -> Config:
        return Config(n, c.DataDir)
    return opt


def WithDataDir(path: str):  # db.go:75-82
    def opt(c: Config) -> Config:
        return Config(c.MaxDataFileSize, path)
    return opt


def Open(dbPath: str, *opts, device: int = 0):
    """gocask.Open: Disk FS unless dbPath == InMemoryDB; defaults 10 GiB files
    under ~/gcdata (db.go:29-59).  Returns (db, err); db is None on error."""
    cfg = Config(10 * GB, os.path.join(os.path.expanduser("~"), "gcdata"))
    for o in opts:
        cfg = o(cfg)
    fs = NewInMemory() if dbPath == InMemoryDB else NewDisk()
    db, err = NewDB(dbPath, fs, None, cfg, device=device)
    if err is not None:
        return None, err
    return db, None


# ---------------------------------------------------------------- replay API
def _files_struct(files, reset_after):
    arrs = [np.ascontiguousarray(np.frombuffer(f, np.uint8) if isinstance(f, (bytes, bytearray)) else f,
                                 dtype=np.uint8) for f in files]
    fa = (GckFile * max(1, len(arrs)))()
    for i, a in enumerate(arrs):
        fa[i].data = a.ctypes.data if a.size else None
        fa[i].len = a.size
        fa[i].reset_after = 1 if reset_after[i] else 0
    return fa, arrs


def _result(res: GckResult):
    n = res.n
    recs = np.zeros(n, dtype=REC_DTYPE)
    if n:
        ctypes.memmove(recs.ctypes.data, res.recs, n * REC_DTYPE.itemsize)
    st = dict(status=res.status, err_file=res.err_file, err_off=res.err_off, n_recs=n,
              n_crc_fail=res.n_crc_fail, final_last_offset=res.final_last_offset,
              files_walked=res.files_walked, n_groups=res.n_groups, n_resident=res.n_resident)
    if res.keys:  # GCK_OPT_KEYS: the records' key bytes back to back
        st["keys"] = np.zeros(res.keys_len, dtype=np.uint8)
        if res.keys_len:
            ctypes.memmove(st["keys"].ctypes.data, res.keys, res.keys_len)
    return recs, st


def host_register(arr):
    """Pin a host numpy buffer (gck_host_register) for DMA-rate transfers."""
    check(_lib.load().gck_host_register(arr.ctypes.data, arr.nbytes))


def host_unregister(arr):
    check(_lib.load().gck_host_unregister(arr.ctypes.data))


def replay(files, reset_after=None, device=0, chunk_bytes=0, max_key=0, chunk_cap=0, spec_window=0,
           max_resident=0, keys=False, live=False):
    """Host-in/host-out replay through gck_replay.  Returns (records, status);
    live=True (GCK_OPT_LIVE): the live keydir records instead of every record."""
    L = _lib.load()
    if reset_after is None:
        reset_after = [True] * len(files)
    fa, arrs = _files_struct(files, reset_after)
    res = GckResult()
    rc = L.gck_replay(fa, len(arrs), ctypes.byref(_opts(device, chunk_bytes, max_key, chunk_cap, spec_window,
                                                        max_resident, keys, live)), ctypes.byref(res))
    try:  # (an error return may still hand back memory: freed either way)
        check(rc, (GCK_OK, GCK_EUNEXPECTED_EOF))
        return _result(res)
    finally:
        L.gck_result_free(ctypes.byref(res))


def replay_hints(hint_files, reset_after=None, device=0, keys=False, live=False):
    """gck_replay_hints: the tuples of the data files behind hint_files (one
    per data file, walk order; reset_after as for the data files) from the
    hints alone.  Returns (records, status); live=True: the keydir (last entry
    per key); keys=True: status["keys"] = the records' key bytes."""
    L = _lib.load()
    if reset_after is None:
        reset_after = [True] * len(hint_files)
    fa, arrs = _files_struct(hint_files, reset_after)
    res = GckResult()
    rc = L.gck_replay_hints(fa, len(arrs), ctypes.byref(_opts(device, 0, 0, 0, 0, 0, keys, live)), ctypes.byref(res))
    try:
        check(rc)
        return _result(res)
    finally:
        L.gck_result_free(ctypes.byref(res))


def replay_paths(paths, reset_after=None, device=0, chunk_bytes=0, max_resident=0, keys=False, live=False):
    """gck_replay_paths: the same replay of files named by path (read by the
    library with pread into page-locked staging buffers).  Returns (records,
    status); live=True (GCK_OPT_LIVE): the live keydir records."""
    L = _lib.load()
    if reset_after is None:
        reset_after = [True] * len(paths)
    enc = [os.fsencode(p) for p in paths]
    pa = (_lib.GckPath * max(1, len(enc)))()
    for i, p in enumerate(enc):
        pa[i].path = p
        pa[i].reset_after = 1 if reset_after[i] else 0
    res = GckResult()
    rc = L.gck_replay_paths(pa, len(enc), ctypes.byref(_opts(device, chunk_bytes, 0, 0, 0, max_resident, keys, live)),
                            ctypes.byref(res))
    try:  # (an error return may still hand back memory: freed either way)
        check(rc, (GCK_OK, GCK_EUNEXPECTED_EOF))
        return _result(res)
    finally:
        L.gck_result_free(ctypes.byref(res))


def replay_into(files, recs, reset_after=None, device=0, chunk_bytes=0, max_resident=0, keys=False, live=False):
    """gck_replay_into: host-in/host-out replay (pipelined over file groups)
    with the tuples written into recs (a REC_DTYPE array; register it with
    host_register for DMA rate).  Returns the status dict; recs[:n] hold the
    records."""
    L = _lib.load()
    if reset_after is None:
        reset_after = [True] * len(files)
    fa, arrs = _files_struct(files, reset_after)
    res = GckResult()
    rc = L.gck_replay_into(fa, len(arrs), ctypes.byref(_opts(device, chunk_bytes, max_resident=max_resident,
                                                             keys=keys, live=live)),
                           recs.ctypes.data if recs.size else None, recs.size, ctypes.byref(res))
    try:
        check(rc, (GCK_OK, GCK_EUNEXPECTED_EOF))
        n, res.n = res.n, 0  # (records are in recs, not in res)
        st = _result(res)[1]
        st["n_recs"] = n
        return st
    finally:
        L.gck_result_free(ctypes.byref(res))


def replay_multi(files, reset_after=None, devices=(0,), chunk_bytes=0, keys=False):
    """gck_replay_multi: the files sharded over `devices` (one rank each), the
    keydir merged across them with RCCL inside the library.  Returns (live
    keydir records, REC_DTYPE with global file indices; status dict, with the
    live entries' key bytes under "keys" when keys=True)."""
    L = _lib.load()
    if reset_after is None:
        reset_after = [True] * len(files)
    fa, arrs = _files_struct(files, reset_after)
    devs = np.ascontiguousarray(devices, dtype=np.int32)
    res = GckResult()
    rc = L.gck_replay_multi(fa, len(arrs), devs.ctypes.data, len(devs),
                            ctypes.byref(_opts(int(devs[0]), chunk_bytes, keys=keys)), ctypes.byref(res))
    try:  # (an error return may still hand back memory: freed either way)
        check(rc, (GCK_OK, GCK_EUNEXPECTED_EOF))
        return _result(res)
    finally:
        L.gck_result_free(ctypes.byref(res))


def replay_multi_paths(paths, reset_after=None, devices=(0,), chunk_bytes=0, keys=False):
    """gck_replay_multi_paths: replay_multi of files named by path."""
    L = _lib.load()
    if reset_after is None:
        reset_after = [True] * len(paths)
    enc = [os.fsencode(p) for p in paths]
    pa = (_lib.GckPath * max(1, len(enc)))()
    for i, p in enumerate(enc):
        pa[i].path = p
        pa[i].reset_after = 1 if reset_after[i] else 0
    devs = np.ascontiguousarray(devices, dtype=np.int32)
    res = GckResult()
    rc = L.gck_replay_multi_paths(pa, len(enc), devs.ctypes.data, len(devs),
                                  ctypes.byref(_opts(int(devs[0]), chunk_bytes, keys=keys)), ctypes.byref(res))
    try:  # (an error return may still hand back memory: freed either way)
        check(rc, (GCK_OK, GCK_EUNEXPECTED_EOF))
        return _result(res)
    finally:
        L.gck_result_free(ctypes.byref(res))


def multi_keydir(ctxs, fetch=True, keys=False):
    """gck_ctx_multi_keydir: the keydir merge of gck_replay_multi over shards
    already resident and replayed in ReplayContexts (ctxs[s] = shard s, walk
    order; one device each, or several on one device: device copies).
    Returns (live records or None, status dict with "n_live" and "ms" =
    keydir + pack, exchange, merge, fetch wall milliseconds; "keys" with
    keys=True)."""
    L = _lib.load()
    hs = (ctypes.c_void_p * max(1, len(ctxs)))(*[c._h.value for c in ctxs])
    res = GckResult()
    ms = (ctypes.c_double * 4)()
    flags = (_lib.MULTI_FETCH if fetch else 0) | (_lib.MULTI_KEYS if keys else 0)
    rc = L.gck_ctx_multi_keydir(hs, len(ctxs), flags, ctypes.byref(res), ms)
    try:
        check(rc, (GCK_OK, GCK_EUNEXPECTED_EOF))
        n = res.n
        if not fetch:
            res.n = 0
        recs, st = _result(res)
        st["n_live"] = n
        st["ms"] = dict(keydir_pack=ms[0], exchange=ms[1], merge=ms[2], fetch=ms[3])
        return (recs if fetch else None), st
    finally:
        res.n = 0
        L.gck_result_free(ctypes.byref(res))


OUTCOME_DTYPE = np.dtype([("status", "<i4"), ("nfiles", "<u4"), ("err_file", "<u4"), ("files_walked", "<u4"),
                          ("final_last_offset", "<u4"), ("_pad", "<u4"), ("err_off", "<u8"), ("n_crc_fail", "<u8")])


def multi_resolve(outcomes, nfiles):
    """gck_replay_multi's global outcome (libgocask_diag.so, host only):
    outcomes = per shard dicts (status, nfiles, err_file, files_walked,
    final_last_offset, err_off, n_crc_fail) in walk order.  Returns (status
    dict, contributes per shard)."""
    D = _lib.load_diag()
    a = np.zeros(max(1, len(outcomes)), dtype=OUTCOME_DTYPE)
    for i, o in enumerate(outcomes):
        for k, v in o.items():
            a[i][k] = v
    contrib = np.zeros(max(1, len(outcomes)), dtype=np.uint8)
    res = GckResult()
    check(D.gck_diag_multi_resolve(a.ctypes.data, len(outcomes), nfiles, ctypes.byref(res), contrib.ctypes.data))
    st = dict(status=res.status, err_file=res.err_file, err_off=res.err_off, n_crc_fail=res.n_crc_fail,
              final_last_offset=res.final_last_offset, files_walked=res.files_walked)
    return st, [bool(x) for x in contrib[:len(outcomes)]]


def multi_recv_offsets(counts):
    """The exchange's receive layout (libgocask_diag.so, host only): counts
    [nsrc][nown] -> offsets [nown][nsrc + 1]."""
    D = _lib.load_diag()
    c = np.ascontiguousarray(counts, dtype=np.uint64)
    nsrc, nown = c.shape
    off = np.zeros((nown, nsrc + 1), dtype=np.uint64)
    check(D.gck_diag_multi_recv_offsets(c.ctypes.data if c.size else None, nsrc, nown, off.ctypes.data))
    return off


def replay_multi_loopback(files, reset_after=None, nshards=2, device=0, chunk_bytes=0, max_resident=0, keys=False):
    """gck_replay_multi's orchestration with nshards logical shards on one
    device, the partitions moved by device copies (libgocask_diag.so test
    entry): the same plan, ring replays, keydir packs, status resolution,
    receive layout and per-owner merges as the N-GPU call."""
    D = _lib.load_diag()
    L = _lib.load()
    if reset_after is None:
        reset_after = [True] * len(files)
    fa, arrs = _files_struct(files, reset_after)
    res = GckResult()
    rc = D.gck_diag_replay_multi_loopback(fa, len(arrs), nshards, device,
                                          ctypes.byref(_opts(device, chunk_bytes, max_resident=max_resident, keys=keys)),
                                          ctypes.byref(res))
    try:  # (an error return may still hand back memory: freed either way)
        check(rc, (GCK_OK, GCK_EUNEXPECTED_EOF))
        return _result(res)
    finally:
        L.gck_result_free(ctypes.byref(res))


def plan_shards(sizes, reset_after, world):
    """gck_plan_shards (host only): [(a, b), ...] file ranges per shard."""
    L = _lib.load()
    sz = np.ascontiguousarray(sizes, dtype=np.uint64)
    rs = np.ascontiguousarray([1 if r else 0 for r in reset_after], dtype=np.uint8)
    out = np.zeros(2 * world, dtype=np.uint32)
    check(L.gck_plan_shards(sz.ctypes.data if sz.size else None, rs.ctypes.data if rs.size else None, len(sz), world,
                            out.ctypes.data))
    return [(int(out[2 * r]), int(out[2 * r + 1])) for r in range(world)]


def release_cache():
    """gck_replay_release_cache: free the device contexts gck_replay keeps."""
    _lib.load().gck_replay_release_cache()


def keydir(files, recs):
    """Apply the tuples in walk order (core/keydir.go:22-49): {key: record row}."""
    kd = {}
    for r in recs:
        f = files[int(r["file"])]
        o = int(r["rec_off"]) + 16
        key = bytes(f[o:o + int(r["key_len"])])
        if int(r["flags"]) & F_TOMBSTONE:
            kd.pop(key, None)
        else:
            kd[key] = r
    return kd


class ReplayContext:
    """Device-resident replay (gck_ctx_*): load or encode once, run many times."""

    def __init__(self, device=0, chunk_bytes=0, max_key=0, chunk_cap=0, spec_window=0):
        self._L = _lib.load()
        self._h = ctypes.c_void_p()
        self._n_live = 0
        check(self._L.gck_ctx_create(ctypes.byref(_opts(device, chunk_bytes, max_key, chunk_cap, spec_window)),
                                     ctypes.byref(self._h)))

    def load(self, files, reset_after=None):
        if reset_after is None:
            reset_after = [True] * len(files)
        fa, arrs = _files_struct(files, reset_after)
        check(self._L.gck_ctx_load(self._h, fa, len(arrs)))

    def encode(self, **kw):
        """Encode a synthetic corpus on the device (gck_encode_corpus)."""
        c = GckCorpusCfg()
        d = dict(seed=1, max_file_size=64 * MB, n_ops=0, n_files=1, key_min=16, key_max=16, key_universe=0,
                 val_fixed=1024, tomb_permille=0, flip_permille=0, ts_base=1700000000, key_seed=0)
        d.update(kw)
        for k, v in d.items():
            setattr(c, k, v)
        nf = ctypes.c_uint32()
        nops = ctypes.c_uint64()
        sizes = np.zeros(1 << 16, dtype=np.uint64)
        check(self._L.gck_encode_corpus(self._h, ctypes.byref(c), ctypes.byref(nf), ctypes.byref(nops),
                                        sizes.ctypes.data, sizes.size))
        order = np.zeros(nf.value, dtype=np.uint32)
        self._L.gck_encode_walk_order(self._h, order.ctypes.data, nf.value)
        return dict(n_files=nf.value, n_ops=nops.value, sizes=sizes[:nf.value].copy(), walk_order=order)

    def encode_files(self, file_ids, last_is_active=False, **kw):
        """One-file corpora data_<id>_... (seed = seed + id), in the given
        (walk) order, into the arena (gck_encode_files): BASELINE C4's shards."""
        c = GckCorpusCfg()
        d = dict(seed=1, max_file_size=64 * MB, n_ops=0, n_files=1, key_min=16, key_max=16, key_universe=0,
                 val_fixed=1024, tomb_permille=0, flip_permille=0, ts_base=1700000000, key_seed=0)
        d.update(kw)
        for k, v in d.items():
            setattr(c, k, v)
        ids = np.ascontiguousarray(file_ids, dtype=np.uint32)
        sizes = np.zeros(max(len(ids), 1), dtype=np.uint64)
        nops = ctypes.c_uint64()
        check(self._L.gck_encode_files(self._h, ctypes.byref(c), ids.ctypes.data, len(ids), 1 if last_is_active else 0,
                                       ctypes.byref(nops), sizes.ctypes.data))
        return dict(n_files=len(ids), n_ops=nops.value, sizes=sizes[:len(ids)].copy(),
                    walk_order=np.arange(len(ids), dtype=np.uint32), file_ids=ids.copy())

    def run(self):
        return check(self._L.gck_ctx_run(self._h), (GCK_OK, GCK_EUNEXPECTED_EOF))

    def fetch(self):
        res = GckResult()
        check(self._L.gck_ctx_fetch(self._h, ctypes.byref(res)))
        try:
            return _result(res)
        finally:
            self._L.gck_result_free(ctypes.byref(res))

    def fetch_into(self, recs):
        """Tuples of the last run into a REC_DTYPE array (gck_ctx_fetch_into);
        returns the number of records."""
        n = ctypes.c_uint64()
        check(self._L.gck_ctx_fetch_into(self._h, recs.ctypes.data, recs.size, ctypes.byref(n)))
        return n.value

    def keydir_hash(self, on=True):
        """gck_ctx_keydir_hash: the next runs hash every record's key in their
        finalize pass, so keydir() reads no key bytes to hash them."""
        check(self._L.gck_ctx_keydir_hash(self._h, 1 if on else 0))

    def keydir(self, keep_tombstones=False, fetch=True):
        """Device keydir of the last run (gck_ctx_keydir + gck_ctx_fetch_keydir):
        (live REC_DTYPE records in walk order, device ms); with fetch=False
        (entry count, device ms) and the entries stay on the device."""
        n, ms = ctypes.c_uint64(), ctypes.c_double()
        check(self._L.gck_ctx_keydir(self._h, 1 if keep_tombstones else 0, ctypes.byref(n), ctypes.byref(ms)))
        self._n_live = n.value
        if not fetch:
            return n.value, ms.value
        recs = np.zeros(n.value, dtype=REC_DTYPE)
        got = ctypes.c_uint64()
        check(self._L.gck_ctx_fetch_keydir(self._h, recs.ctypes.data if n.value else None, n.value,
                                           ctypes.byref(got)))
        return recs, ms.value

    # -- merge (compaction) and hint files (include/gocask_hip.h) --
    def compact(self, max_file_size, fetch=True):
        """Merge the live records of the device keydir (keydir() first, without
        tombstones) into new data files + hint files (gck_ctx_compact): with
        fetch, (list of data-file bytes, list of hint-file bytes, device ms);
        else (files, data bytes, hint bytes, device ms), outputs on the device."""
        nf, nd, nh, ms = ctypes.c_uint32(), ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_double()
        check(self._L.gck_ctx_compact(self._h, int(max_file_size), ctypes.byref(nf), ctypes.byref(nd),
                                      ctypes.byref(nh), ctypes.byref(ms)))
        if not fetch:
            return nf.value, nd.value, nh.value, ms.value
        data = np.zeros(max(nd.value, 1), dtype=np.uint8)
        hints = np.zeros(max(nh.value, 1), dtype=np.uint8)
        fsz = np.zeros(max(nf.value, 1), dtype=np.uint64)
        hsz = np.zeros(max(nf.value, 1), dtype=np.uint64)
        check(self._L.gck_ctx_fetch_compact(self._h, data.ctypes.data, fsz.ctypes.data, hints.ctypes.data,
                                            hsz.ctypes.data))
        files, hfiles, a, b = [], [], 0, 0
        for k in range(nf.value):
            files.append(data[a:a + int(fsz[k])].copy())
            hfiles.append(hints[b:b + int(hsz[k])].copy())
            a += int(fsz[k])
            b += int(hsz[k])
        return files, hfiles, ms.value

    def replay_hints(self):
        """Hint-driven replay of the hint files loaded into this context
        (gck_ctx_replay_hints): the tuples a run of their data files gives,
        flags F_HINT, from the hints alone.  Returns the device ms; fetch() /
        keydir() then work as after run()."""
        ms = ctypes.c_double()
        check(self._L.gck_ctx_replay_hints(self._h, ctypes.byref(ms)))
        return ms.value

    # -- batched Get / scrub (include/gocask_hip.h) --
    def get_batch(self, keys, values=True):
        """DB.Get for every key against the device keydir (keydir() first):
        (status int32[n], value_size u32[n], crc_calc u32[n], values list or
        None); values[i] is bytes for GCK_OK keys, else None."""
        n = len(keys)
        off = np.zeros(n + 1, dtype=np.uint64)
        off[1:] = np.cumsum([len(k) for k in keys], dtype=np.uint64)
        blob = np.frombuffer(b"".join(bytes(k) for k in keys) or b"\0", dtype=np.uint8)
        st = np.zeros(n, dtype=np.int32)
        vs = np.zeros(n, dtype=np.uint32)
        cc = np.zeros(n, dtype=np.uint32)
        ms = ctypes.c_double()
        if not values:
            check(self._L.gck_ctx_get_batch(self._h, blob.ctypes.data, off.ctypes.data, n, st.ctypes.data,
                                            vs.ctypes.data, cc.ctypes.data, None, 0, None, ctypes.byref(ms)))
            self.last_get_ms = ms.value
            return st, vs, cc, None
        vo = np.zeros(n, dtype=np.uint64)
        cap = 1 << 20
        while True:
            buf = np.zeros(cap, dtype=np.uint8)
            rc = self._L.gck_ctx_get_batch(self._h, blob.ctypes.data, off.ctypes.data, n, st.ctypes.data,
                                           vs.ctypes.data, cc.ctypes.data, buf.ctypes.data, cap, vo.ctypes.data,
                                           ctypes.byref(ms))
            need = int(vs[st == GCK_OK].sum(dtype=np.uint64))
            if rc == GCK_EINVAL and need > cap:
                cap = need
                continue
            check(rc)
            break
        vals = [bytes(buf[int(vo[i]):int(vo[i]) + int(vs[i])]) if st[i] == GCK_OK else None for i in range(n)]
        self.last_get_ms = ms.value  # device time of the lookup, CRCs and value copy (events)
        return st, vs, cc, vals

    def scrub_keydir(self):
        """Get of every live keydir entry on the device: (status int32[n_live],
        crc_calc u32[n_live], n_bad, device ms)."""
        st = np.zeros(self._n_live, dtype=np.int32)
        cc = np.zeros(self._n_live, dtype=np.uint32)
        bad, ms = ctypes.c_uint64(), ctypes.c_double()
        check(self._L.gck_ctx_scrub_keydir(self._h, st.ctypes.data if st.size else None,
                                           cc.ctypes.data if cc.size else None, ctypes.byref(bad), ctypes.byref(ms)))
        return st, cc, bad.value, ms.value

    # -- keydir merge across shards (include/gocask_hip.h) --
    def kd_pack_sizes(self, nparts):
        """After keydir(keep_tombstones=True): (entries, key bytes) per owner."""
        cnt = (ctypes.c_uint64 * nparts)()
        kb = (ctypes.c_uint64 * nparts)()
        check(self._L.gck_kd_pack_sizes(self._h, nparts, cnt, kb))
        return list(cnt), list(kb)

    def kd_pack(self, shard, file_base, d_entries, entries_cap, d_keys, keys_cap):
        """Fill device buffers (raw pointers) with the partitioned entries / keys."""
        check(self._L.gck_kd_pack(self._h, shard, file_base, d_entries, entries_cap, d_keys, keys_cap))

    def kd_merge(self, d_entries, d_keys, src_counts, src_key_bytes):
        """Merge received partitions (device pointers, sources in shard order):
        (live entries, device ms)."""
        ns = len(src_counts)
        cnt = (ctypes.c_uint64 * ns)(*src_counts)
        kb = (ctypes.c_uint64 * ns)(*src_key_bytes)
        n, ms = ctypes.c_uint64(), ctypes.c_double()
        check(self._L.gck_kd_merge(self._h, d_entries, d_keys, cnt, kb, ns, ctypes.byref(n), ctypes.byref(ms)))
        return n.value, ms.value

    def kd_fetch_merged(self):
        """Host copies of the merged entries (KD_ENTRY_DTYPE) and their key blob."""
        n, nk = ctypes.c_uint64(), ctypes.c_uint64()
        check(self._L.gck_kd_fetch_merged(self._h, None, 0, None, 0, ctypes.byref(n), ctypes.byref(nk)))
        ents = np.zeros(n.value, dtype=KD_ENTRY_DTYPE)
        keys = np.zeros(nk.value, dtype=np.uint8)
        check(self._L.gck_kd_fetch_merged(self._h, ents.ctypes.data if n.value else None, n.value,
                                          keys.ctypes.data if nk.value else None, nk.value, ctypes.byref(n),
                                          ctypes.byref(nk)))
        return ents, keys

    def stats(self):
        s = GckStats()
        check(self._L.gck_ctx_stats(self._h, ctypes.byref(s)))
        phases = {}
        for i in range(12):
            name = self._L.gck_phase_name(i).decode()
            if not name:
                break
            phases[name] = s.ms_kernel[i]
        return dict(bytes=s.bytes, n_recs=s.n_recs, n_crc_fail=s.n_crc_fail, n_chunks=s.n_chunks,
                    n_fixups=s.n_fixups, n_overflow=s.n_overflow, ms_total=s.ms_total, ms_phase=phases,
                    device_path=bool(s.device_path), n_reruns=s.n_reruns, status=s.status, err_file=s.err_file,
                    err_off=s.err_off, files_walked=s.files_walked, final_last_offset=s.final_last_offset,
                    n_files=s.n_files, n_runs=s.n_runs, ms_crc_rows_sum=s.ms_crc_rows_sum,
                    kd_longest_probe=s.kd_longest_probe)

    def phase_timing(self, on=True):
        """Events between every phase of the next runs (stats()['ms_phase'] per
        phase).  Off (the default): a device-path run times only the CRC pass
        (ms_phase 'crc_rows'; the other phases and 'pipeline' read 0, since an
        event between two kernels costs ~6 us of the run); a host-path run
        (a context's first) always times every phase."""
        check(self._L.gck_ctx_phase_timing(self._h, 1 if on else 0))

    def stream_read_ceiling(self, iters=10):
        """Plain streaming read of the resident arena (measurement helper,
        libgocask_diag.so): (ms per pass, GB/s)."""
        ms = ctypes.c_double()
        gbs = ctypes.c_double()
        check(_lib.load_diag().gck_diag_stream_read(self._h, iters, ctypes.byref(ms), ctypes.byref(gbs)))
        return ms.value, gbs.value

    def stream_blocks_ceiling(self, iters=10, static_eighths=4, stamp=False):
        """The XCD-balanced stream ceiling (measurement helper,
        libgocask_diag.so): k_crc_rows' geometry and work assignment -- 64-row
        blocks, half static, half from an atomic queue -- without its compute.
        (ms per pass, GB/s); stamp: the last pass leaves per-wavefront clock
        stamps for clock_stamps()."""
        ms = ctypes.c_double()
        gbs = ctypes.c_double()
        check(_lib.load_diag().gck_diag_stream_blocks(self._h, iters, static_eighths, int(bool(stamp)),
                                                      ctypes.byref(ms), ctypes.byref(gbs)))
        return ms.value, gbs.value

    def stream_xp(self, pf=1, blocks=True, threads=1024, lds_kib=160, wg_per_cu=1, iters=10, stamp=False):
        """Stream probe (libgocask_diag.so gck_diag_stream_xp): k_crc_rows' row
        loads with pf rows in flight per wavefront and no compute; blocks 0:
        rows strided over the wavefronts, 1: static 64-row blocks (block
        k W + w), 2: every block from an atomic queue, 3: k_crc_rows' split
        (half the full rounds static, the rest queued); occupancy from the
        workgroup size, its LDS and workgroups per CU.  (ms per pass, GB/s);
        stamp: see clock_stamps()."""
        ms = ctypes.c_double()
        gbs = ctypes.c_double()
        check(_lib.load_diag().gck_diag_stream_xp(self._h, pf, int(blocks), threads, lds_kib, wg_per_cu, iters,
                                                  int(bool(stamp)), ctypes.byref(ms), ctypes.byref(gbs)))
        return ms.value, gbs.value

    def stream_rows_ceiling(self, iters=10, stamp=False):
        """The balanced stream ceiling over k_crc_rows' rows: its load pattern
        (a wavefront per 4 KiB row, 16 B per lane, non-temporal) in whole
        64-row blocks, half of them static and the rest from one queue per
        XCD, 4 wavefronts per CU with 3 rows in flight each, no compute.  Of
        the round-6 probes (tools/stream_xp.py, profiles/r6r) the fastest
        whose wavefronts end together (4.83-4.84 ms for C3, the last wave
        within 0.03 ms of the median; static blocks stream in 4.78-4.90 ms
        but their median wave ends 0.2-1.3 ms before the last)."""
        return self.stream_xp(3, 6, 256, 160, 1, iters, stamp)

    @staticmethod
    def clock_stamps():
        """(stamps u64[W, 4] = clock, real time at start; clock, real time at
        end; xcc u32[W]) of the last stamped stream_blocks_ceiling / stream_xp pass."""
        w = 16384
        st = np.zeros(4 * w, dtype=np.uint64)
        xcc = np.zeros(w, dtype=np.uint32)
        check(_lib.load_diag().gck_diag_clock_read(st.ctypes.data, xcc.ctypes.data, w))
        return st.reshape(w, 4), xcc

    def read_file(self, file, off=0, length=None, out=None):
        n = length
        buf = np.zeros(n, dtype=np.uint8) if out is None else out
        if n:
            check(self._L.gck_ctx_read_file(self._h, file, off, buf.ctypes.data, n))
        return buf

    def close(self):
        if self._h:
            self._L.gck_ctx_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def zipf_table():
    t = np.zeros(65472, dtype=np.uint32)
    _lib.load().gck_encode_zipf_table(t.ctypes.data)
    return t


def device_count():
    return _lib.load().gck_device_count()


def encode_batch(ops, device="cuda"):
    """Bulk serializeEntry on the device (row f4, `gck_encode_batch`).

    ops: iterable of (ts, key, value) -- value None means a Delete of key.
    Returns the serialized bytes as a uint8 torch tensor on `device`, and the
    record offsets (n+1, int64 tensor), exactly as DB.Put / DB.Delete append
    them (core/db.go:185-212, :245-247, serializeEntry :272-284)."""
    import torch

    ops = list(ops)
    n = len(ops)
    keys = b"".join(k for _, k, _ in ops)
    vals = b"".join(v for _, _, v in ops if v is not None)
    koff = np.zeros(n + 1, dtype=np.uint64)
    voff = np.zeros(n + 1, dtype=np.uint64)
    koff[1:] = np.cumsum([len(k) for _, k, _ in ops], dtype=np.uint64) if n else koff[1:]
    voff[1:] = np.cumsum([0 if v is None else len(v) for _, _, v in ops], dtype=np.uint64) if n else voff[1:]
    ts = np.array([t & 0xFFFFFFFF for t, _, _ in ops], dtype=np.uint32)
    tomb = np.array([v is None for _, _, v in ops], dtype=np.uint8)

    def dev(a, dtype):
        return torch.from_numpy(np.array(a, copy=True).view(dtype)).to(device)

    # the kernel reads whole dwords: up to 4 bytes past a blob's end (header)
    d_keys = dev(np.frombuffer(keys + bytes(16), dtype=np.uint8), np.uint8)
    d_vals = dev(np.frombuffer(vals + bytes(16), dtype=np.uint8), np.uint8)
    d_koff, d_voff = dev(koff, np.int64), dev(voff, np.int64)
    d_ts, d_tomb = dev(ts, np.int32), dev(tomb, np.uint8)
    need = int(16 * n + len(keys) + sum(len(v) for _, _, v in ops if v is not None))
    out = torch.empty(max(need, 1), dtype=torch.uint8, device=device)
    out_off = torch.empty(n + 1, dtype=torch.int64, device=device)
    total = ctypes.c_uint64(0)
    stream = torch.cuda.current_stream(out.device).cuda_stream
    _lib.check(_lib.load().gck_encode_batch(d_keys.data_ptr(), d_koff.data_ptr(), d_vals.data_ptr(),
                                            d_voff.data_ptr(), d_ts.data_ptr(), d_tomb.data_ptr(), n,
                                            out.data_ptr(), out.numel(), out_off.data_ptr(),
                                            ctypes.byref(total), stream))
    return out[: total.value], out_off
