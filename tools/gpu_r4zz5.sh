set -o pipefail
out=gpurun_out/r4zz5
mkdir -p $out
L=gocask_amd/var
bash tools/ab_mix.sh 2 $L/libgocask_hip_head.so $L/libgocask_hip_so24.so $L/libgocask_hip_so16.so $L/libgocask_hip_so8.so > $out/ab_spec_occ.log 2>&1 || { cat $out/ab_spec_occ.log; exit 1; }
cut -c1-200 $out/ab_spec_occ.log
