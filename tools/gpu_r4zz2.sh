set -o pipefail
out=gpurun_out/r4zz2
mkdir -p $out
L=gocask_amd/var
bash tools/ab_mix.sh 3 $L/libgocask_hip_head.so $L/libgocask_hip_specdef.so > $out/ab_spec_policy.log 2>&1 || { cat $out/ab_spec_policy.log; exit 1; }
cut -c1-250 $out/ab_spec_policy.log
