"""gocask_amd — MI355X-native cold-start replay for GoCask data files.

The product is libgocask_hip.so (C-ABI, include/gocask_hip.h): HIP kernels for
gfx950 plus a C++ host mirror of core.NewDB / gocask.Open.  This package is the
thin ctypes layer over it (the Python counterpart of a cgo stub).
"""
from .core import (GB, KB, MB, TB, Config, DB, DefaultConfig, ErrCRCFailed, ErrInvalidKey, ErrInvalidValue,
                   ErrKeyNotFound, ErrPartialWrite, ErrUnexpectedEOF, GoCaskError, InMemoryDB, NewDB, NewDisk,
                   NewInMemory, Open, ReplayContext, StartupError, WithDataDir, WithMaxDataFileSize, device_count,
                   host_register, host_unregister, keydir, plan_shards, release_cache, replay, replay_into, replay_paths,
                   replay_multi, replay_multi_paths, zipf_table, multi_resolve, multi_recv_offsets,
                   replay_multi_loopback, multi_keydir, replay_hints)
from ._lib import F_CRC_OK, F_HINT, F_TOMBSTONE, REC_DTYPE

__all__ = [
    "GB", "KB", "MB", "TB", "Config", "DB", "DefaultConfig", "ErrCRCFailed", "ErrInvalidKey", "ErrInvalidValue",
    "ErrKeyNotFound", "ErrPartialWrite", "ErrUnexpectedEOF", "GoCaskError", "InMemoryDB", "NewDB", "NewDisk",
    "NewInMemory", "Open", "ReplayContext", "StartupError", "WithDataDir", "WithMaxDataFileSize", "device_count",
    "host_register", "host_unregister", "keydir", "plan_shards", "release_cache", "replay", "replay_into", "replay_paths",
    "replay_multi", "replay_multi_paths", "zipf_table", "multi_resolve", "multi_recv_offsets", "replay_multi_loopback", "multi_keydir", "replay_hints",
    "F_CRC_OK", "F_HINT", "F_TOMBSTONE", "REC_DTYPE",
]
