set -o pipefail
out=gpurun_out/r4zx
mkdir -p $out
L=gocask_amd/var
bash tools/scrub_ab.sh $L/libgocask_hip_head.so $L/libgocask_hip_ver8.so $L/libgocask_hip_ver12.so > $out/scrub_ab.log 2>&1 || { cat $out/scrub_ab.log; exit 1; }
cat $out/scrub_ab.log
bash tools/ab_mix.sh 2 $L/libgocask_hip_head.so $L/libgocask_hip_crc8.so $L/libgocask_hip_crc12.so > $out/ab_crc_waves.log 2>&1 || { cat $out/ab_crc_waves.log; exit 1; }
cut -c1-160 $out/ab_crc_waves.log
