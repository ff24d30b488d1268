# Round 4 final measurement set on the shipped build
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r4final
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $out/gpu_suite.log 2>&1
rc=$?
tail -3 $out/gpu_suite.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { cat $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 300 python bench.py > $out/bench_default.json 2> $out/bench_default.err || { tail -20 $out/bench_default.err; exit 1; }
cat $out/bench_default.json
bash tools/pmc.sh r4final || exit $?
for rep in 1 2; do
  GCK_LIB_PATH=gocask_amd/var/libgocask_hip_clk.so timeout -k 10 150 python tools/clock.py >> $out/clock.log 2>&1 || exit $?
done
grep '^{' $out/clock.log | cut -c1-400
