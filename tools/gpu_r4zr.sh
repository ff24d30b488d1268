set -o pipefail
out=gpurun_out/r4zr
mkdir -p $out
L=gocask_amd/var
for v in claim ntall; do
  GCK_LIB_PATH=$L/libgocask_hip_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_encode_batch.py -m gpu -x -q --timeout 200 --timeout-method thread > $out/pytest_$v.log 2>&1 || { tail -5 $out/pytest_$v.log; exit 1; }
  tail -1 $out/pytest_$v.log
done
bash tools/enc_ab.sh $L/libgocask_hip_ntst.so $L/libgocask_hip_claim.so $L/libgocask_hip_ntall.so > $out/enc_ab.log 2>&1 || { cat $out/enc_ab.log; exit 1; }
bash tools/enc_ab.sh $L/libgocask_hip_ntst.so $L/libgocask_hip_claim.so $L/libgocask_hip_ntall.so >> $out/enc_ab.log 2>&1 || { cat $out/enc_ab.log; exit 1; }
cut -c1-200 $out/enc_ab.log
