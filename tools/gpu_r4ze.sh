set -o pipefail
out=gpurun_out/r4ze
mkdir -p $out
GCK_LIB_PATH=gocask_amd/var/libgocask_hip_encdiag3.so timeout -k 10 200 python tools/bench_encode.py > $out/encdiag3.log 2>&1 || { tail $out/encdiag3.log; exit 1; }
grep -E "ENCDIAG3|GBps" $out/encdiag3.log | tail -3 | cut -c1-200
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/kt -o kt -- python tools/bench_encode.py > $out/kt.log 2>&1 || { tail $out/kt.log; exit 1; }
find $out/kt -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $out/enc_kernel_stats.csv
cut -d, -f1-8 $out/enc_kernel_stats.csv | head -8
