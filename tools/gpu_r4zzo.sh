set -o pipefail
out=gpurun_out/r4zzo
mkdir -p $out
L=gocask_amd/var
GCK_LIB_PATH=$L/libgocask_hip_fq.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_configs.py -m gpu -x -q --timeout 400 --timeout-method thread > $out/pytest.log 2>&1 || { tail -15 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
bash tools/ab_mix.sh 3 $L/libgocask_hip_head.so $L/libgocask_hip_fq.so > $out/ab_fin_queue.log 2>&1 || { cat $out/ab_fin_queue.log; exit 1; }
cut -c1-250 $out/ab_fin_queue.log
