set -o pipefail
out=gpurun_out/r4w
mkdir -p $out
GCK_LIB_PATH=gocask_amd/var/libgocask_hip_encdiag.so timeout -k 10 200 python tools/bench_encode.py > $out/encdiag.log 2>&1 || { tail $out/encdiag.log; exit 1; }
grep -E "ENCDIAG|GBps" $out/encdiag.log | tail -4
