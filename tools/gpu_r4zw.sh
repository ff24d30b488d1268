set -o pipefail
out=gpurun_out/r4zw
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_encode_batch.py tests/test_gpu_compact.py -m gpu -x -q --timeout 200 --timeout-method thread > $out/pytest.log 2>&1 || { tail -5 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
L=gocask_amd/var
bash tools/enc_ab.sh $L/libgocask_hip_w8.so $L/libgocask_hip_lb512.so $L/libgocask_hip_lb512r8.so > $out/enc_ab.log 2>&1 || { cat $out/enc_ab.log; exit 1; }
cut -c1-200 $out/enc_ab.log
