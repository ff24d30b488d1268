set -o pipefail
out=gpurun_out/r4zy
mkdir -p $out
L=gocask_amd/var
bash tools/scrub_ab.sh $L/libgocask_hip_head.so $L/libgocask_hip_snt0.so $L/libgocask_hip_snt0w12.so > $out/scrub_ab.log 2>&1 || { cat $out/scrub_ab.log; exit 1; }
bash tools/scrub_ab.sh $L/libgocask_hip_head.so $L/libgocask_hip_snt0.so $L/libgocask_hip_snt0w12.so >> $out/scrub_ab.log 2>&1 || { cat $out/scrub_ab.log; exit 1; }
cat $out/scrub_ab.log
