set -o pipefail
out=gpurun_out/r4zb
mkdir -p $out
L=gocask_amd/var
bash tools/scrub_ab.sh $L/libgocask_hip_base.so $L/libgocask_hip_al64.so > $out/scrub_ab.log 2>&1 || { cat $out/scrub_ab.log; exit 1; }
bash tools/scrub_ab.sh $L/libgocask_hip_base.so $L/libgocask_hip_al64.so >> $out/scrub_ab.log 2>&1 || { cat $out/scrub_ab.log; exit 1; }
cat $out/scrub_ab.log
bash tools/enc_ab.sh $L/libgocask_hip_base.so $L/libgocask_hip_al64.so > $out/enc_ab.log 2>&1 || { cat $out/enc_ab.log; exit 1; }
cut -c1-200 $out/enc_ab.log
GCK_LIB_PATH=gocask_amd/var/libgocask_hip_encdiag2.so timeout -k 10 200 python tools/bench_encode.py > $out/encdiag2.log 2>&1 || { tail $out/encdiag2.log; exit 1; }
grep -E "ENCDIAG2|GBps" $out/encdiag2.log | tail -3
