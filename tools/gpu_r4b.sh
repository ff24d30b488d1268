# Round 4: full GPU suite on the tree with the multi-GPU ring + loopback work,
# then the r2-vs-HEAD interleaved A/B + in-kernel clock stamps.
set -o pipefail
mkdir -p gpurun_out/r4b
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread \
  > gpurun_out/r4b/pytest.log 2>&1
rc=$?
tail -15 gpurun_out/r4b/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/ab_r2.sh abr2 3 > gpurun_out/r4b/ab.log 2>&1
rc2=$?
cat gpurun_out/r4b/ab.log
exit $((rc ? rc : rc2))
