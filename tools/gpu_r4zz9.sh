set -o pipefail
out=gpurun_out/r4zz9
mkdir -p $out
L=gocask_amd/var
bash tools/ab_mix.sh 2 $L/libgocask_hip_head.so $L/libgocask_hip_cp16.so $L/libgocask_hip_cp32.so > $out/ab_compact_occ.log 2>&1 || { cat $out/ab_compact_occ.log; exit 1; }
cut -c1-250 $out/ab_compact_occ.log
