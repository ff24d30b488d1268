set -o pipefail
out=gpurun_out/r4zg
mkdir -p $out
GCK_LIB_PATH=gocask_amd/var/libgocask_hip_encdiag4.so timeout -k 10 200 python tools/bench_encode.py > $out/encdiag4.log 2>&1 || { tail $out/encdiag4.log; exit 1; }
grep -E "ENCDIAG4|GBps" $out/encdiag4.log | tail -3 | cut -c1-200
bash tools/enc_kt.sh gocask_amd/libgocask_hip.so > $out/enc_kt.log 2>&1 || { cat $out/enc_kt.log; exit 1; }
cat $out/enc_kt.log
cp gpurun_out/enckt_1/bench.log $out/enc_kt_bench.log
