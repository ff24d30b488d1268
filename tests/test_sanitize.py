"""ASan + UBSan builds of the host code (the reference's
`go test -race`, Makefile:3), CPU only: the oracle and the C++ host mirror
(gocask_amd/csrc/db.cpp: walk, path, mmap, keydir fill, Get) replay every
golden fixture and the Open/Get/Keys disk cases under the sanitizers
(tests/sanitize/run_san.py).  Any sanitizer report fails the test."""
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
SAN = os.path.join(HERE, "sanitize")


def _libasan():
    try:
        p = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True, check=True)
    except (OSError, subprocess.CalledProcessError):
        return None
    path = p.stdout.strip()
    return path if os.path.isabs(path) and os.path.exists(path) else None


def test_host_code_under_asan_ubsan():
    asan = _libasan()
    if asan is None:
        pytest.skip("gcc's libasan is not available")
    subprocess.run(["make", "-s", "-C", SAN], check=True)
    env = dict(os.environ, LD_PRELOAD=asan,
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:halt_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    p = subprocess.run([sys.executable, os.path.join(SAN, "run_san.py")], env=env, capture_output=True, text=True,
                       timeout=600)
    out = p.stdout + p.stderr
    assert p.returncode == 0, out[-4000:]
    assert "runtime error" not in out and "AddressSanitizer" not in out, out[-4000:]
    assert "oracle ok" in p.stdout and "host ok" in p.stdout
