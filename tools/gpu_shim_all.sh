# shim parity tests, then the C3 Open timing of every shim mode
set -o pipefail
out=gpurun_out/${1:-shim}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_shim.py -m gpu -x -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
timeout -k 10 900 python tools/shim_c3.py 2 > $out/shim_c3.jsonl 2> $out/shim_c3.err || { tail -20 $out/shim_c3.err; exit 1; }
python3 -c "
import json
for l in open('$out/shim_c3.jsonl'):
    d=json.loads(l); print(d['mode'], 'multi' if d['multi'] else 'single', d['rep'], d['records'], d['walk_mmap_register_ms'], d['replay_ms'], d['unregister_unmap_ms'], d['open_ms'])
"
