set -o pipefail
out=gpurun_out/r4zj
mkdir -p $out
L=gocask_amd/var
bash tools/enc_ab.sh $L/libgocask_hip_encln.so $L/libgocask_hip_lm128.so $L/libgocask_hip_lm64.so $L/libgocask_hip_ring8.so > $out/enc_ab.log 2>&1 || { cat $out/enc_ab.log; exit 1; }
cut -c1-200 $out/enc_ab.log
bash tools/scrub_ab.sh $L/libgocask_hip_encln.so $L/libgocask_hip_ring8.so > $out/scrub_ab.log 2>&1 || { cat $out/scrub_ab.log; exit 1; }
cat $out/scrub_ab.log
