set -o pipefail
out=gpurun_out/r4zzm
mkdir -p $out
L=gocask_amd/var
bash tools/enc_ab.sh $L/libgocask_hip_head.so $L/libgocask_hip_u32k.so $L/libgocask_hip_u128k.so > $out/enc_ab.log 2>&1 || { cat $out/enc_ab.log; exit 1; }
bash tools/enc_ab.sh $L/libgocask_hip_head.so $L/libgocask_hip_u32k.so $L/libgocask_hip_u128k.so >> $out/enc_ab.log 2>&1 || { cat $out/enc_ab.log; exit 1; }
cut -c1-170 $out/enc_ab.log
