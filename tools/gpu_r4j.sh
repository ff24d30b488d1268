set -o pipefail
out=gpurun_out/r4j
mkdir -p $out
export GCK_REPLAY_TRACE=1 SHIM_MODES="4 0"
timeout -k 10 600 python tools/shim_c3.py 3 > $out/shim_c3.jsonl 2> $out/shim_c3.err || { tail -20 $out/shim_c3.err; exit 1; }
python3 -c "
import json
for l in open('$out/shim_c3.jsonl'):
    d=json.loads(l); print(d['mode'], d['multi'], d['rep'], d['open_ms']); print('\n'.join(d.get('trace',[])))
"
