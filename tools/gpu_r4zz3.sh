set -o pipefail
out=gpurun_out/r4zz3
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_encode_batch.py -m gpu -x -v --timeout 300 --timeout-method thread > $out/pytest.log 2>&1 || { tail -15 $out/pytest.log; exit 1; }
grep -E "random_large|passed" $out/pytest.log | tail -4
