set -o pipefail
out=gpurun_out/r4o
mkdir -p $out
L=gocask_amd/var
bash tools/scrub_ab.sh gocask_amd/libgocask_hip.so $L/libgocask_hip_static.so $L/libgocask_hip_noboth.so $L/libgocask_hip_noboth_static.so $L/libgocask_hip_noboth_nofill.so > $out/scrub_ablate2.log 2>&1 || { cat $out/scrub_ablate2.log; exit 1; }
cat $out/scrub_ablate2.log
