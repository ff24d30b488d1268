set -o pipefail
out=gpurun_out/r4k
mkdir -p $out
bash tools/ab_mix.sh 3 gocask_amd/var/libgocask_hip_base.so gocask_amd/var/libgocask_hip_xi.so > $out/ab_xi.log 2>&1
rc=$?
cat $out/ab_xi.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $out/pytest.log 2>&1
rc=$?
tail -3 $out/pytest.log
exit $rc
