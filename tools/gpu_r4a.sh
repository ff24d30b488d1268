# Round 4, first GPU call: the bench self-launch test, then the r2-vs-HEAD A/B + clocks.
set -o pipefail
mkdir -p gpurun_out/r4a
timeout -k 10 300 python -u -m pytest tests/test_bench_launch.py -x -v --timeout 280 --timeout-method thread -m gpu \
  > gpurun_out/r4a/launch.log 2>&1
rc=$?
tail -5 gpurun_out/r4a/launch.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/ab_r2.sh abr2 3 > gpurun_out/r4a/ab.log 2>&1
rc2=$?
cat gpurun_out/r4a/ab.log
exit $((rc2 ? rc2 : rc))
