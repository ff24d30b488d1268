# GPU suite on this build, then the C3 Open timing of the shim's modes
set -o pipefail
out=gpurun_out/${1:-r3w}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/gpu_suite.log 2>&1 || { tail -40 $out/gpu_suite.log; exit 1; }
tail -2 $out/gpu_suite.log
timeout -k 10 600 python tools/shim_c3.py 2 > $out/shim_c3.jsonl 2> $out/shim_c3.err || { tail -20 $out/shim_c3.err; exit 1; }
cat $out/shim_c3.jsonl
