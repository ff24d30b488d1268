"""Host-inclusive Open of the C3 workload as the cgo shim pays it
(tests/shim/shim_test.c in SHIM_TIME mode): the 16 x 2 GiB
files written to /dev/shm (page cache, as a warm database directory), then
the shim walks, stats, mmaps and gck_host_register's every file inside the
Walk callback, calls gck_replay (or gck_replay_multi on device 0), frees the
tuples, unregisters and unmaps.  One JSON line per run; the directory is
removed at the end.  Modes: by path (gck_replay_paths: the library preads the
files into its staging buffers), pageable mappings (staged by the library),
pinned mappings (the shim registers each mmap), pinned + gck_replay_multi,
by path + gck_replay_multi, by path with GCK_OPT_LIVE (mode 5: the live
keydir instead of every record).  Every mode includes the shim's keydir map
fill (map_fill.cpp, a C++ unordered_map as the Go map's proxy).
python tools/shim_c3.py [reps] [number of modes]"""
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import gocask_amd as g  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
d = "/dev/shm/gck_c3"
shutil.rmtree(d, ignore_errors=True)
os.makedirs(d)
try:
    with g.ReplayContext() as ctx:
        info = ctx.encode(**bench.CONFIGS["c3"])
        for w in range(info["n_files"]):
            n = int(info["walk_order"][w])
            size = int(info["sizes"][n])
            buf = ctx.read_file(w, 0, size)
            with open(os.path.join(d, f"data_{n}_{1700000000 + n}.csk"), "wb") as f:
                f.write(buf.tobytes())
            del buf
    shim = os.path.join(ROOT, "tests", "shim", "build", "shim_test")
    out = []
    modes = [dict(SHIM_PATHS="1"), dict(SHIM_PIN="0"), dict(SHIM_PIN="1"), dict(SHIM_PIN="1", SHIM_MULTI="1"),
             dict(SHIM_PATHS="1", SHIM_MULTI="1"), dict(SHIM_PATHS="1", SHIM_LIVE="1"),
             dict(SHIM_PATHS="1", SHIM_LIVE="1", GCK_STAGE_HOSTMALLOC="1")]  # (6: staging by hipHostMalloc, an A/B)
    if len(sys.argv) > 2:
        modes = modes[:int(sys.argv[2])]
    if os.environ.get("SHIM_MODES"):  # e.g. "0 4": by path, single and multi
        modes = [modes[int(i)] for i in os.environ["SHIM_MODES"].split()]
    # SHIM_THREADS="4 8 16": the by-path / pageable modes at each copy-thread count
    threads = os.environ.get("SHIM_THREADS", "").split()
    if threads:
        modes = [dict(m, GCK_COPY_THREADS=t) for t in threads for m in modes if m.get("SHIM_PIN") != "1"]
    # SHIM_AB_DIRS="dir1 dir2": each mode with the libgocask_hip.so of each directory, interleaved
    libdirs = os.environ.get("SHIM_AB_DIRS", "").split() or [None]
    runs = [(m, r, ld) for r in range(reps) for m in modes for ld in libdirs]  # (modes interleaved)
    for mode, r, ld in runs:
        if True:
            env = dict(os.environ, SHIM_TIME="1", **mode)
            if ld:
                env["LD_LIBRARY_PATH"] = os.path.abspath(ld) + ":" + env.get("LD_LIBRARY_PATH", "")
            p = subprocess.run([shim, d], capture_output=True, text=True, timeout=300, env=env)
            if p.returncode:
                raise SystemExit(p.stderr)
            row = json.loads(p.stdout.strip().splitlines()[-1])
            row["rep"] = r
            row["libdir"] = ld
            row["stage_hostmalloc"] = "GCK_STAGE_HOSTMALLOC" in mode
            row["copy_threads"] = mode.get("GCK_COPY_THREADS", os.environ.get("GCK_COPY_THREADS", "default"))
            tr = [l for l in p.stderr.splitlines() if l.startswith(("gck_replay", "[gck_replay"))]
            if tr:  # GCK_REPLAY_TRACE=1: the library's phase marks
                row["trace"] = tr
            out.append(row)
            print(json.dumps(row), flush=True)
finally:
    shutil.rmtree(d, ignore_errors=True)
