set -o pipefail
out=gpurun_out/r4u
mkdir -p $out
L=gocask_amd/var
bash tools/scrub_ab.sh gocask_amd/libgocask_hip.so $L/libgocask_hip_lane0.so $L/libgocask_hip_lane64.so > $out/scrub_lane.log 2>&1 || { cat $out/scrub_lane.log; exit 1; }
cat $out/scrub_lane.log
