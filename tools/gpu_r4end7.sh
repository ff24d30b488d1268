# Round 4 end-of-round measurement set on the shipped build (encoder rebuilt)
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r4end7
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $out/gpu_suite.log 2>&1
rc=$?
tail -3 $out/gpu_suite.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { cat $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 300 python bench.py > $out/bench_default.json 2> $out/bench_default.err || { tail -20 $out/bench_default.err; exit 1; }
cat $out/bench_default.json
bash tools/pmc.sh r4end7 || exit $?
bash tools/enc_kt.sh gocask_amd/libgocask_hip.so > $out/enc_kt.log 2>&1 || { cat $out/enc_kt.log; exit 1; }
cat $out/enc_kt.log
cp gpurun_out/enckt_1/run_kernel_stats.csv $out/enc_kernel_stats.csv
for rep in 1 2 3; do timeout -k 10 120 python tools/bench_encode.py 2>/dev/null | tail -1 >> $out/bench_encode.log || exit 1; done
cut -c1-200 $out/bench_encode.log
for rep in 1 2 3; do timeout -k 10 150 python tools/scrub.py 2>/dev/null | tail -1 >> $out/scrub.log || exit 1; done
cat $out/scrub.log
for rep in 1 2; do timeout -k 10 300 python tools/bench_get.py 2>/dev/null | tail -1 >> $out/bench_get.log || exit 1; done
cat $out/bench_get.log
for rep in 1 2; do timeout -k 10 300 python tools/bench_compact.py 2>/dev/null | tail -1 >> $out/bench_compact.log || exit 1; done
cut -c1-220 $out/bench_compact.log
