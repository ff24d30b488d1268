set -o pipefail
out=gpurun_out/r4zz6
mkdir -p $out
L=gocask_amd/var
bash tools/scrub_ab.sh $L/libgocask_hip_head.so $L/libgocask_hip_ring2.so $L/libgocask_hip_ring8.so > $out/scrub_ab.log 2>&1 || { cat $out/scrub_ab.log; exit 1; }
bash tools/scrub_ab.sh $L/libgocask_hip_head.so $L/libgocask_hip_ring2.so $L/libgocask_hip_ring8.so >> $out/scrub_ab.log 2>&1 || { cat $out/scrub_ab.log; exit 1; }
cat $out/scrub_ab.log
bash tools/enc_ab.sh $L/libgocask_hip_head.so $L/libgocask_hip_ring2.so $L/libgocask_hip_ring8.so > $out/enc_ab.log 2>&1 || { cat $out/enc_ab.log; exit 1; }
cut -c1-160 $out/enc_ab.log
