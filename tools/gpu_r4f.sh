set -o pipefail
mkdir -p gpurun_out/r4f
bash tools/ab_mix.sh 3 abr2 abh . > gpurun_out/r4f/ab.log 2>&1
rc=$?
cat gpurun_out/r4f/ab.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r4f/pytest.log 2>&1
rc=$?
tail -5 gpurun_out/r4f/pytest.log
[ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  GCK_LIB_PATH=gocask_amd/var/libgocask_hip_clk.so timeout -k 10 150 python tools/clock.py >> gpurun_out/r4f/clock.log 2>&1 || exit $?
done
grep '^{' gpurun_out/r4f/clock.log
