set -o pipefail
out=gpurun_out/r4zz8
mkdir -p $out
L=gocask_amd/var
bash tools/ab_mix.sh 2 $L/libgocask_hip_head.so $L/libgocask_hip_fin2.so $L/libgocask_hip_fin3.so $L/libgocask_hip_fin4.so > $out/ab_fin_blocks.log 2>&1 || { cat $out/ab_fin_blocks.log; exit 1; }
cut -c1-250 $out/ab_fin_blocks.log
