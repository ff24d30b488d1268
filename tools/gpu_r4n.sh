# Scrub and encoder ablations (where the time goes), interleaved
set -o pipefail
out=gpurun_out/r4n
mkdir -p $out
L=gocask_amd/var
bash tools/scrub_ab.sh gocask_amd/libgocask_hip.so $L/libgocask_hip_nolane.so $L/libgocask_hip_nowave.so $L/libgocask_hip_noboth.so > $out/scrub_ablate.log 2>&1 || { cat $out/scrub_ablate.log; exit 1; }
cat $out/scrub_ablate.log
bash tools/enc_ab.sh gocask_amd/libgocask_hip.so $L/libgocask_hip_enc_nocrc.so $L/libgocask_hip_enc_nocopy.so > $out/enc_ablate.log 2>&1 || { cat $out/enc_ablate.log; exit 1; }
cat $out/enc_ablate.log
