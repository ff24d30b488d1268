"""C-ABI boundary checks that need no GPU: the library builds, loads, exports
every symbol include/gocask_hip.h declares, host-only helpers agree with the
oracle, and compute entry points fail loudly (no CPU fallback) without a device.
"""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "gocask_hip.h")


@pytest.fixture(scope="module")
def lib():
    import __graft_entry__

    __graft_entry__.build()
    import gocask_amd

    return gocask_amd._lib.load()


def declared_symbols():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(gck_\w+)\s*\(", txt)))


def test_header_declares_entry_points():
    syms = declared_symbols()
    assert "gck_replay" in syms and "gck_db_open" in syms and "gck_ctx_run" in syms
    import gocask_amd._lib as L

    assert sorted(L.EXPORTED) == syms


def test_library_exports_every_declared_symbol(lib):
    so = os.path.join(ROOT, "gocask_amd", "libgocask_hip.so")
    out = subprocess.run(["nm", "-D", "--defined-only", so], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r" T (gck_\w+)", out))
    missing = [s for s in declared_symbols() if s not in exported]
    assert not missing, missing
    for s in declared_symbols():
        assert hasattr(lib, s)


def test_library_targets_gfx950_only():
    so = os.path.join(ROOT, "gocask_amd", "libgocask_hip.so")
    data = open(so, "rb").read()
    assert b"gfx950" in data
    assert b"gfx942" not in data and b"gfx90a" not in data


def test_abi_struct_layouts():
    import gocask_amd._lib as L

    assert L.REC_DTYPE.itemsize == 40
    assert ctypes.sizeof(L.GckFile) == 24
    assert ctypes.sizeof(L.GckResult) == 72  # + keys, keys_len (GCK_OPT_KEYS)
    assert ctypes.sizeof(L.GckPath) == 16
    assert ctypes.sizeof(L.GckOpts) == 32
    assert ctypes.sizeof(L.GckCorpusCfg) == 72


def test_encoder_zipf_table_matches_oracle(lib, orc):
    import gocask_amd as g

    assert np.array_equal(g.zipf_table(), orc.zipf_table())


def test_no_cpu_fallback_without_device(lib):
    import gocask_amd as g

    if g.device_count() > 0:
        pytest.skip("a GPU is present; covered by -m gpu tests")
    with pytest.raises(g._lib.GckError) as e:
        g.replay([b"\x00" * 16])
    assert e.value.code == g._lib.GCK_EDEVICE
    db = None
    with pytest.raises(g._lib.GckError):
        db, _ = g.NewDB("", g.NewInMemory(b""))
    assert db is None
