set -o pipefail
out=gpurun_out/r3y
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_paths.py tests/test_gpu_ring.py tests/test_gpu_shim.py tests/test_gpu_parity.py tests/test_gpu_multi.py -m gpu -x -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -2 $out/tests.log
SHIM_THREADS="16" GCK_REPLAY_TRACE=1 timeout -k 10 600 python tools/shim_c3.py 3 1 > $out/shim_trace.jsonl 2> $out/shim_trace.err || { tail -20 $out/shim_trace.err; exit 1; }
python3 -c "
import json
for l in open('$out/shim_trace.jsonl'):
    d=json.loads(l); print(d['mode'], d['copy_threads'], d['rep'], d['replay_ms'], d['open_ms']); print('\n'.join(d.get('trace',[])[:2]+d.get('trace',[])[-2:]))
"
