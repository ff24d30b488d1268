# Round 4 measurement call: default bench, kernel trace + PMC passes, counter list
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r4g
mkdir -p $out
timeout -k 10 300 python bench.py > $out/bench_default.json 2> $out/bench_default.err || { tail -20 $out/bench_default.err; exit 1; }
cat $out/bench_default.json
timeout -k 10 60 rocprofv3 -L > $out/counters.txt 2>&1 || true
bash tools/pmc.sh r4g || exit $?
