set -o pipefail
mkdir -p gpurun_out/r4e
bash tools/ab_mix.sh 3 abr2 gocask_amd/var/libgocask_hip_nomb.so . > gpurun_out/r4e/ab.log 2>&1
rc=$?
cat gpurun_out/r4e/ab.log
exit $rc
