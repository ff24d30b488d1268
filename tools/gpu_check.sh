#!/bin/bash
# One GPU call: the -m gpu suite, smoke, and a default bench line.
#   bash tools/gpu_check.sh <tag> [pytest -k expr]   -> gpurun_out/<tag>/
set -o pipefail
tag=${1:-chk}; kexpr=${2:-}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
if [ -n "$kexpr" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$kexpr" > $out/gpu_suite.log 2>&1 || { tail -30 $out/gpu_suite.log; exit 1; }
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/gpu_suite.log 2>&1 || { tail -30 $out/gpu_suite.log; exit 1; }
fi
tail -3 $out/gpu_suite.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { cat $out/smoke.log; exit 1; }
cat $out/smoke.log | tail -1
timeout -k 10 300 python bench.py > $out/bench_default.json 2> $out/bench.err || { tail $out/bench.err; exit 1; }
python3 -c "
import json,sys; d=json.loads(open('$out/bench_default.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['crc_rows_ms'], d['phase_ms'], d['cpu_baseline']['value'])"
