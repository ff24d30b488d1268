# Round 4 call c: the GPU tests the first call did not reach (-x stopped at a
# test bug), the new full-size CRC/timestamp flip test, smoke; then the
# r2 / HEAD-orig / bitfield-cap A/B.
set -o pipefail
mkdir -p gpurun_out/r4c
timeout -k 10 900 python -u -m pytest tests/test_gpu_paths.py tests/test_gpu_ring.py tests/test_gpu_shim.py \
  tests/test_gpu_fuzz.py -m gpu -x -v -s --timeout 400 --timeout-method thread -k "not test_bit_flips_anywhere" \
  > gpurun_out/r4c/pytest.log 2>&1
rc=$?
grep -E "PASS|FAIL|ERROR|c3 file|passed|failed" gpurun_out/r4c/pytest.log | tail -40
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4c/smoke.log 2>&1 || exit $?
cat gpurun_out/r4c/smoke.log
bash tools/ab_trees.sh 3 abr2 abh . > gpurun_out/r4c/ab.log 2>&1
rc2=$?
cat gpurun_out/r4c/ab.log
[ $rc2 -ne 0 ] && exit $rc2
for rep in 1 2; do
  GCK_LIB_PATH=gocask_amd/var/libgocask_hip_clk.so timeout -k 10 150 python tools/clock.py >> gpurun_out/r4c/clock.log 2>&1 || exit $?
done
grep '^{' gpurun_out/r4c/clock.log
exit $rc
