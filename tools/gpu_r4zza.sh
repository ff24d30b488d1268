set -o pipefail
out=gpurun_out/r4zza
mkdir -p $out
L=gocask_amd/var
GCK_LIB_PATH=$L/libgocask_hip_r64.so timeout -k 10 300 python -u -m pytest tests/test_gpu_encode_batch.py tests/test_gpu_get.py -m gpu -x -q --timeout 200 --timeout-method thread > $out/pytest.log 2>&1 || { tail -5 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
bash tools/enc_ab.sh $L/libgocask_hip_head.so $L/libgocask_hip_r64.so > $out/enc_ab.log 2>&1 || { cat $out/enc_ab.log; exit 1; }
cut -c1-200 $out/enc_ab.log
bash tools/scrub_ab.sh $L/libgocask_hip_head.so $L/libgocask_hip_r64.so > $out/scrub_ab.log 2>&1 || { cat $out/scrub_ab.log; exit 1; }
bash tools/scrub_ab.sh $L/libgocask_hip_head.so $L/libgocask_hip_r64.so >> $out/scrub_ab.log 2>&1 || { cat $out/scrub_ab.log; exit 1; }
cat $out/scrub_ab.log
