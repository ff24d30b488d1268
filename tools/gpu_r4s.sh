set -o pipefail
out=gpurun_out/r4s
mkdir -p $out
L=gocask_amd/var
bash tools/scrub_ab.sh $L/libgocask_hip_noboth.so $L/libgocask_hip_nb_nolds.so > $out/scrub_ablate4.log 2>&1 || { cat $out/scrub_ablate4.log; exit 1; }
cat $out/scrub_ablate4.log
