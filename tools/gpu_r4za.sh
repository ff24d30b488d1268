set -o pipefail
out=gpurun_out/r4za
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_get.py tests/test_gpu_encode_batch.py tests/test_gpu_compact.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?
tail -2 $out/pytest.log
[ $rc -ne 0 ] && exit $rc
L=gocask_amd/var
bash tools/scrub_ab.sh $L/libgocask_hip_base.so $L/libgocask_hip_z5.so > $out/scrub_ab.log 2>&1 || { cat $out/scrub_ab.log; exit 1; }
bash tools/scrub_ab.sh $L/libgocask_hip_base.so $L/libgocask_hip_z5.so >> $out/scrub_ab.log 2>&1 || { cat $out/scrub_ab.log; exit 1; }
cat $out/scrub_ab.log
bash tools/enc_ab.sh $L/libgocask_hip_base.so $L/libgocask_hip_z5.so > $out/enc_ab.log 2>&1 || { cat $out/enc_ab.log; exit 1; }
cut -c1-200 $out/enc_ab.log
