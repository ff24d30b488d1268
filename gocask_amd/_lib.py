"""ctypes binding of libgocask_hip.so (include/gocask_hip.h).

This is the Python equivalent of the cgo stub a Go maintainer would add
(INTEGRATION.md).  It loads the in-tree library and fails loudly when it is
missing: there is no CPU fallback for the replay path.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GCK_LIB_PATH") or os.path.join(HERE, "libgocask_hip.so")

GCK_OK = 0
GCK_EUNEXPECTED_EOF = 1
GCK_EDEVICE = 2
GCK_EINVAL = 3
GCK_ENOMEM = 4
GCK_EIO = 5
GCK_EKEY_NOT_FOUND = 6
GCK_ECRC_FAILED = 7
GCK_EINVALID_KEY = 8
GCK_ENOT_DIR = 9


F_TOMBSTONE = 1
F_CRC_OK = 2
F_HINT = 4  # from a hint file (gck_ctx_replay_hints): value not read
HINT_BLOCK, HINT_MAGIC, HINT_VERSION = 16, 0x484B4347, 3  # GCK_HINT_*

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
assert REC_DTYPE.itemsize == 40

# gck_kd_entry: one keydir entry crossing shards (include/gocask_hip.h)
KD_ENTRY_DTYPE = np.dtype([("hash", "<u8"), ("key_off", "<u8"), ("key_len", "<u4"), ("shard", "<u4"),
                           ("rec", REC_DTYPE)])
assert KD_ENTRY_DTYPE.itemsize == 64

# Every symbol include/gocask_hip.h declares (tests check the .so exports them).
EXPORTED = [
    "gck_replay", "gck_replay_into", "gck_replay_paths", "gck_result_free", "gck_replay_release_cache", "gck_ctx_create", "gck_ctx_destroy", "gck_ctx_load", "gck_ctx_run", "gck_ctx_phase_timing",
    "gck_ctx_fetch", "gck_ctx_fetch_into", "gck_ctx_keydir", "gck_ctx_keydir_hash", "gck_ctx_fetch_keydir", "gck_ctx_get_batch", "gck_ctx_scrub_keydir", "gck_ctx_compact", "gck_ctx_fetch_compact", "gck_ctx_replay_hints", "gck_replay_hints", "gck_kd_pack_sizes", "gck_kd_pack", "gck_kd_merge", "gck_kd_fetch_merged", "gck_replay_multi", "gck_replay_multi_paths", "gck_ctx_multi_keydir", "gck_plan_shards", "gck_ctx_stats", "gck_phase_name", "gck_ctx_device_recs", "gck_ctx_stream",
    "gck_ctx_read_file", "gck_encode_corpus", "gck_encode_files", "gck_encode_walk_order", "gck_encode_zipf_table", "gck_encode_batch", "gck_db_open",
    "gck_db_open_mem", "gck_db_get", "gck_db_keys", "gck_db_key", "gck_db_entry", "gck_db_last_offset",
    "gck_db_active_file", "gck_db_nfiles", "gck_db_file_name", "gck_db_close", "gck_device_count", "gck_host_register", "gck_host_unregister",
    "gck_version", "gck_last_error",
]


OPT_KEYS = 1  # gck_opts.flags GCK_OPT_KEYS
OPT_LIVE = 2  # gck_opts.flags GCK_OPT_LIVE
MULTI_FETCH, MULTI_KEYS = 1, 2  # gck_ctx_multi_keydir flags


class GckFile(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p), ("len", ctypes.c_uint64), ("reset_after", ctypes.c_uint8)]


class GckPath(ctypes.Structure):
    _fields_ = [("path", ctypes.c_char_p), ("reset_after", ctypes.c_uint8)]


class GckOpts(ctypes.Structure):
    _fields_ = [
        ("device", ctypes.c_int32),
        ("chunk_bytes", ctypes.c_uint32),
        ("max_key", ctypes.c_uint32),
        ("chunk_cap", ctypes.c_uint32),
        ("flags", ctypes.c_uint32),
        ("spec_window", ctypes.c_uint32),
        ("max_resident", ctypes.c_uint64),
    ]


class GckResult(ctypes.Structure):
    _fields_ = [
        ("recs", ctypes.c_void_p),
        ("n", ctypes.c_uint64),
        ("n_crc_fail", ctypes.c_uint64),
        ("final_last_offset", ctypes.c_uint32),
        ("status", ctypes.c_int32),
        ("err_file", ctypes.c_uint32),
        ("files_walked", ctypes.c_uint32),
        ("err_off", ctypes.c_uint64),
        ("n_groups", ctypes.c_uint32),
        ("n_resident", ctypes.c_uint32),
        ("keys", ctypes.c_void_p),
        ("keys_len", ctypes.c_uint64),
    ]


class GckStats(ctypes.Structure):
    _fields_ = [
        ("bytes", ctypes.c_uint64),
        ("n_recs", ctypes.c_uint64),
        ("n_crc_fail", ctypes.c_uint64),
        ("n_chunks", ctypes.c_uint64),
        ("n_fixups", ctypes.c_uint64),
        ("n_overflow", ctypes.c_uint64),
        ("ms_total", ctypes.c_double),
        ("ms_kernel", ctypes.c_double * 12),
        ("device_path", ctypes.c_uint32),
        ("n_reruns", ctypes.c_uint32),
        ("status", ctypes.c_int32),
        ("err_file", ctypes.c_uint32),
        ("err_off", ctypes.c_uint64),
        ("files_walked", ctypes.c_uint32),
        ("final_last_offset", ctypes.c_uint32),
        ("n_files", ctypes.c_uint32),
        ("kd_longest_probe", ctypes.c_uint32),
        ("n_runs", ctypes.c_uint64),
        ("ms_crc_rows_sum", ctypes.c_double),
    ]


class GckCorpusCfg(ctypes.Structure):
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
    ]


class GckConfig(ctypes.Structure):
    _fields_ = [("max_data_file_size", ctypes.c_int64), ("data_dir", ctypes.c_char_p)]


_lib = None
_diag = None
DIAG_PATH = os.environ.get("GCK_DIAG_PATH") or os.path.join(HERE, "libgocask_diag.so")


def _torch_runtime_first():
    """torch ships its own HIP runtime (libamdhip64 + ROCr from its wheel) next
    to the system one this library links; in one process torch's only comes up
    if it initialises first ("No HIP GPUs are available" otherwise).  The
    Python host side uses torch for device buffers and torch.distributed (the
    keydir exchange), so let it initialise before the first call into
    libgocask_hip.  A process without torch is unaffected."""
    try:
        import torch
    except ImportError:
        return
    try:
        if torch.cuda.is_available():
            torch.cuda.init()
    except Exception:  # torch without a usable device: the library reports its own errors
        pass


def load():
    """Load the in-tree HIP library.  Raises if it has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} missing: run __graft_entry__.build() (no CPU fallback exists)")
    _torch_runtime_first()
    L = ctypes.CDLL(LIB_PATH)
    P = ctypes.POINTER
    vp = ctypes.c_void_p
    sig = {
        "gck_replay": (ctypes.c_int, [P(GckFile), ctypes.c_uint32, P(GckOpts), P(GckResult)]),
        "gck_replay_into": (ctypes.c_int, [P(GckFile), ctypes.c_uint32, P(GckOpts), vp, ctypes.c_uint64, P(GckResult)]),
        "gck_replay_paths": (ctypes.c_int, [P(GckPath), ctypes.c_uint32, P(GckOpts), P(GckResult)]),
        "gck_result_free": (None, [P(GckResult)]),
        "gck_replay_release_cache": (None, []),
        "gck_ctx_create": (ctypes.c_int, [P(GckOpts), P(vp)]),
        "gck_ctx_destroy": (None, [vp]),
        "gck_ctx_load": (ctypes.c_int, [vp, P(GckFile), ctypes.c_uint32]),
        "gck_ctx_run": (ctypes.c_int, [vp]),
        "gck_ctx_phase_timing": (ctypes.c_int, [vp, ctypes.c_int]),
        "gck_ctx_fetch": (ctypes.c_int, [vp, P(GckResult)]),
        "gck_ctx_fetch_into": (ctypes.c_int, [vp, vp, ctypes.c_uint64, P(ctypes.c_uint64)]),
        "gck_ctx_keydir": (ctypes.c_int, [vp, ctypes.c_uint32, P(ctypes.c_uint64), P(ctypes.c_double)]),
        "gck_ctx_fetch_keydir": (ctypes.c_int, [vp, vp, ctypes.c_uint64, P(ctypes.c_uint64)]),
        "gck_ctx_keydir_hash": (ctypes.c_int, [vp, ctypes.c_int]),
        "gck_ctx_get_batch": (ctypes.c_int, [vp, vp, vp, ctypes.c_uint32, vp, vp, vp, vp, ctypes.c_uint64, vp,
                                             P(ctypes.c_double)]),
        "gck_ctx_scrub_keydir": (ctypes.c_int, [vp, vp, vp, P(ctypes.c_uint64), P(ctypes.c_double)]),
        "gck_ctx_compact": (ctypes.c_int, [vp, ctypes.c_uint64, P(ctypes.c_uint32), P(ctypes.c_uint64),
                                           P(ctypes.c_uint64), P(ctypes.c_double)]),
        "gck_ctx_fetch_compact": (ctypes.c_int, [vp, vp, vp, vp, vp]),
        "gck_ctx_replay_hints": (ctypes.c_int, [vp, P(ctypes.c_double)]),
        "gck_replay_hints": (ctypes.c_int, [P(GckFile), ctypes.c_uint32, P(GckOpts), P(GckResult)]),
        "gck_kd_pack_sizes": (ctypes.c_int, [vp, ctypes.c_uint32, P(ctypes.c_uint64), P(ctypes.c_uint64)]),
        "gck_kd_pack": (ctypes.c_int, [vp, ctypes.c_uint32, ctypes.c_uint32, vp, ctypes.c_uint64, vp,
                                       ctypes.c_uint64]),
        "gck_kd_merge": (ctypes.c_int, [vp, vp, vp, P(ctypes.c_uint64), P(ctypes.c_uint64), ctypes.c_uint32,
                                        P(ctypes.c_uint64), P(ctypes.c_double)]),
        "gck_kd_fetch_merged": (ctypes.c_int, [vp, vp, ctypes.c_uint64, vp, ctypes.c_uint64, P(ctypes.c_uint64),
                                               P(ctypes.c_uint64)]),
        "gck_replay_multi": (ctypes.c_int, [P(GckFile), ctypes.c_uint32, vp, ctypes.c_uint32, P(GckOpts),
                                            P(GckResult)]),
        "gck_replay_multi_paths": (ctypes.c_int, [P(GckPath), ctypes.c_uint32, vp, ctypes.c_uint32, P(GckOpts),
                                                 P(GckResult)]),
        "gck_ctx_multi_keydir": (ctypes.c_int, [vp, ctypes.c_uint32, ctypes.c_uint32, P(GckResult),
                                                P(ctypes.c_double)]),
        "gck_plan_shards": (ctypes.c_int, [vp, vp, ctypes.c_uint32, ctypes.c_uint32, vp]),
        "gck_ctx_stats": (ctypes.c_int, [vp, P(GckStats)]),
        "gck_phase_name": (ctypes.c_char_p, [ctypes.c_int]),
        "gck_ctx_device_recs": (ctypes.c_int, [vp, P(vp), P(ctypes.c_uint64)]),
        "gck_ctx_stream": (vp, [vp]),
        "gck_ctx_read_file": (ctypes.c_int, [vp, ctypes.c_uint32, ctypes.c_uint64, vp, ctypes.c_uint64]),
        "gck_encode_corpus": (ctypes.c_int, [vp, P(GckCorpusCfg), P(ctypes.c_uint32), P(ctypes.c_uint64), vp,
                                             ctypes.c_uint32]),
        "gck_encode_files": (ctypes.c_int, [vp, P(GckCorpusCfg), vp, ctypes.c_uint32, ctypes.c_uint32, vp, vp]),
        "gck_encode_walk_order": (ctypes.c_int, [vp, vp, ctypes.c_uint32]),
        "gck_encode_zipf_table": (None, [vp]),
        "gck_encode_batch": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, ctypes.c_uint64, vp, ctypes.c_uint64, vp,
                                            P(ctypes.c_uint64), vp]),
        "gck_db_open": (ctypes.c_int, [ctypes.c_char_p, P(GckConfig), P(GckOpts), P(vp), ctypes.c_char_p,
                                       ctypes.c_size_t]),
        "gck_db_open_mem": (ctypes.c_int, [vp, ctypes.c_uint64, P(GckOpts), P(vp), ctypes.c_char_p,
                                           ctypes.c_size_t]),
        "gck_db_get": (ctypes.c_int, [vp, ctypes.c_char_p, ctypes.c_uint32, P(vp), P(ctypes.c_uint64)]),
        "gck_db_keys": (ctypes.c_uint64, [vp]),
        "gck_db_key": (ctypes.c_int, [vp, ctypes.c_uint64, P(vp), P(ctypes.c_uint32)]),
        "gck_db_entry": (ctypes.c_int, [vp, ctypes.c_char_p, ctypes.c_uint32, P(ctypes.c_uint32),
                                        P(ctypes.c_uint32), P(ctypes.c_uint32), P(ctypes.c_uint32),
                                        P(ctypes.c_char_p)]),
        "gck_db_last_offset": (ctypes.c_uint32, [vp]),
        "gck_db_active_file": (ctypes.c_char_p, [vp]),
        "gck_db_nfiles": (ctypes.c_uint32, [vp]),
        "gck_db_file_name": (ctypes.c_char_p, [vp, ctypes.c_uint32]),
        "gck_db_close": (None, [vp]),
        "gck_device_count": (ctypes.c_int, []),
        "gck_host_register": (ctypes.c_int, [vp, ctypes.c_uint64]),
        "gck_host_unregister": (ctypes.c_int, [vp]),
        "gck_version": (ctypes.c_char_p, []),
        "gck_last_error": (ctypes.c_char_p, []),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def load_diag():
    """The measurement helpers (gocask_amd/csrc/gck_diag.h), a separate
    library linked against libgocask_hip.so; not part of the product ABI."""
    global _diag
    if _diag is not None:
        return _diag
    load()
    if not os.path.exists(DIAG_PATH):
        raise ImportError(f"{DIAG_PATH} missing: run __graft_entry__.build()")
    D = ctypes.CDLL(DIAG_PATH)
    P = ctypes.POINTER
    vp = ctypes.c_void_p
    D.gck_diag_stream_read.restype = ctypes.c_int
    D.gck_diag_stream_read.argtypes = [vp, ctypes.c_int, P(ctypes.c_double), P(ctypes.c_double)]
    D.gck_diag_stream_pattern.restype = ctypes.c_int
    D.gck_diag_stream_pattern.argtypes = [vp, ctypes.c_int, ctypes.c_int, P(ctypes.c_double), P(ctypes.c_double)]
    D.gck_diag_stream_blocks.restype = ctypes.c_int
    D.gck_diag_stream_blocks.argtypes = [vp, ctypes.c_int, ctypes.c_uint32, ctypes.c_int, P(ctypes.c_double),
                                         P(ctypes.c_double)]
    if hasattr(D, "gck_diag_stream_xp"):  # (diag libraries of older builds, for A/Bs, lack it)
        D.gck_diag_stream_xp.restype = ctypes.c_int
        D.gck_diag_stream_xp.argtypes = [vp] + [ctypes.c_int] * 7 + [P(ctypes.c_double), P(ctypes.c_double)]
    D.gck_diag_clock_read.restype = ctypes.c_int
    D.gck_diag_clock_read.argtypes = [vp, vp, ctypes.c_uint32]
    D.gck_diag_chunks.restype = ctypes.c_int
    D.gck_diag_chunks.argtypes = [vp, vp, vp, ctypes.c_uint64, P(ctypes.c_uint64)]
    D.gck_diag_multi_resolve.restype = ctypes.c_int
    D.gck_diag_multi_resolve.argtypes = [vp, ctypes.c_uint32, ctypes.c_uint32, P(GckResult), vp]
    D.gck_diag_multi_recv_offsets.restype = ctypes.c_int
    D.gck_diag_multi_recv_offsets.argtypes = [vp, ctypes.c_uint32, ctypes.c_uint32, vp]
    D.gck_diag_replay_multi_loopback.restype = ctypes.c_int
    D.gck_diag_replay_multi_loopback.argtypes = [P(GckFile), ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int32,
                                                 P(GckOpts), P(GckResult)]
    _diag = D
    return D


class GckError(RuntimeError):
    def __init__(self, code, msg=""):
        self.code = code
        super().__init__(f"gocask_hip error {code}: {msg}")


def check(rc, allowed=(GCK_OK,)):
    if rc not in allowed:
        L = load()
        raise GckError(rc, (L.gck_last_error() or b"").decode())
    return rc
