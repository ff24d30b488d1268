set -o pipefail
out=gpurun_out/r4zm
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_encode_batch.py tests/test_gpu_compact.py -m gpu -x -v --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?
tail -4 $out/pytest.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" $out/pytest.log | head -20; exit $rc; }
L=gocask_amd/var
bash tools/enc_ab.sh $L/libgocask_hip_enc1rt.so $L/libgocask_hip_encwide.so > $out/enc_ab.log 2>&1 || { cat $out/enc_ab.log; exit 1; }
bash tools/enc_ab.sh $L/libgocask_hip_enc1rt.so $L/libgocask_hip_encwide.so >> $out/enc_ab.log 2>&1 || { cat $out/enc_ab.log; exit 1; }
cut -c1-220 $out/enc_ab.log
