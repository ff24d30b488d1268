set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r5b
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_live.py tests/test_gpu_shim.py tests/test_bench_launch.py tests/test_gpu_ring.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
bash tools/ktrace.sh r5b > $out/kt.log 2>&1 || { tail -20 $out/kt.log; exit 1; }
python3 tools/timeline.py gpurun_out/kt_r5b > $out/timeline.json || exit 1
cat $out/timeline.json
L=gocask_amd/var
bash tools/ab_mix.sh 3 $L/libgocask_hip_base.so gocask_amd/libgocask_hip.so $L/libgocask_hip_st8.so $L/libgocask_hip_eb.so $L/libgocask_hip_gtab.so > $out/ab.log 2>&1 || { cat $out/ab.log; exit 1; }
cut -c1-260 $out/ab.log
GCK_LIB_PATH=gocask_amd/var/libgocask_hip_clk.so timeout -k 10 200 python tools/phase_clock.py > $out/phase_clock.json 2> $out/phase_clock.err || { tail -20 $out/phase_clock.err; exit 1; }
cat $out/phase_clock.json
