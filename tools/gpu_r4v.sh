set -o pipefail
out=gpurun_out/r4v
mkdir -p $out
L=gocask_amd/var
bash tools/scrub_ab.sh $L/libgocask_hip_base.so $L/libgocask_hip_burst.so $L/libgocask_hip_metaburst.so > $out/scrub_ab.log 2>&1 || { cat $out/scrub_ab.log; exit 1; }
bash tools/scrub_ab.sh $L/libgocask_hip_base.so $L/libgocask_hip_burst.so $L/libgocask_hip_metaburst.so >> $out/scrub_ab.log 2>&1 || { cat $out/scrub_ab.log; exit 1; }
cat $out/scrub_ab.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_get.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/test_get.log 2>&1
rc=$?
tail -3 $out/test_get.log
exit $rc
