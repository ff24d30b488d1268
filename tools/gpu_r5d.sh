set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r5d
mkdir -p $out
L=gocask_amd/var
bash tools/ab_mix.sh 3 $L/libgocask_hip_base.so gocask_amd/libgocask_hip.so $L/libgocask_hip_cc2.so $L/libgocask_hip_cc4.so $L/libgocask_hip_eb.so > $out/ab.log 2>&1 || { cat $out/ab.log; exit 1; }
cut -c1-260 $out/ab.log
