set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r5b
mkdir -p $out
bash tools/ktrace.sh r5b > $out/kt.log 2>&1 || { tail -20 $out/kt.log; exit 1; }
python3 tools/timeline.py gpurun_out/kt_r5b > $out/timeline.json || exit 1
cat $out/timeline.json
L=gocask_amd/var
bash tools/ab_mix.sh 3 gocask_amd/libgocask_hip.so $L/libgocask_hip_st8.so $L/libgocask_hip_st6.so $L/libgocask_hip_st2.so $L/libgocask_hip_eb.so > $out/ab.log 2>&1 || { cat $out/ab.log; exit 1; }
cut -c1-260 $out/ab.log
GCK_LIB_PATH=gocask_amd/var/libgocask_hip_clk.so timeout -k 10 200 python tools/phase_clock.py > $out/phase_clock.json 2> $out/phase_clock.err || { tail -20 $out/phase_clock.err; exit 1; }
cat $out/phase_clock.json
timeout -k 10 600 python -u -m pytest tests/test_gpu_live.py tests/test_gpu_shim.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests_live.log 2>&1 || { tail -30 $out/tests_live.log; exit 1; }
tail -2 $out/tests_live.log
