set -o pipefail
out=gpurun_out/r4zv
mkdir -p $out
L=gocask_amd/var
bash tools/enc_ab.sh $L/libgocask_hip_w8.so $L/libgocask_hip_w6.so $L/libgocask_hip_w4.so > $out/enc_ab.log 2>&1 || { cat $out/enc_ab.log; exit 1; }
cut -c1-200 $out/enc_ab.log
