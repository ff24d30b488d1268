set -o pipefail
out=gpurun_out/r4q
mkdir -p $out
L=gocask_amd/var
bash tools/scrub_ab.sh $L/libgocask_hip_noboth.so $L/libgocask_hip_nb_nostore.so $L/libgocask_hip_nb_1grp.so > $out/scrub_ablate3.log 2>&1 || { cat $out/scrub_ablate3.log; exit 1; }
cat $out/scrub_ablate3.log
