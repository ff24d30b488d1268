set -o pipefail
out=gpurun_out/r4y
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $out/pytest.log 2>&1
rc=$?
tail -3 $out/pytest.log
[ $rc -ne 0 ] && exit $rc
GCK_LIB_PATH=gocask_amd/var/libgocask_hip_encdiag.so timeout -k 10 200 python tools/bench_encode.py > $out/encdiag.log 2>&1 || { tail $out/encdiag.log; exit 1; }
grep -E "ENCDIAG|GBps" $out/encdiag.log | tail -2
bash tools/enc_ab.sh gocask_amd/var/libgocask_hip_base.so gocask_amd/var/libgocask_hip_encmask.so > $out/enc_ab.log 2>&1 || { cat $out/enc_ab.log; exit 1; }
cat $out/enc_ab.log
bash tools/ab_mix.sh 3 gocask_amd/var/libgocask_hip_base.so gocask_amd/var/libgocask_hip_valskip.so > $out/ab_valskip.log 2>&1 || { cat $out/ab_valskip.log; exit 1; }
cat $out/ab_valskip.log
