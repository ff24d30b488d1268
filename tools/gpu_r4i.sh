# C3 Open as the shim pays it: by path single-GPU vs the multi-GPU call on device 0 (ring), 3 reps each, trace marks
set -o pipefail
out=gpurun_out/r4i
mkdir -p $out
export GCK_REPLAY_TRACE=1
timeout -k 10 900 python tools/shim_c3.py 3 > $out/shim_c3.jsonl 2> $out/shim_c3.err || { tail -20 $out/shim_c3.err; exit 1; }
python3 -c "
import json
for l in open('$out/shim_c3.jsonl'):
    d=json.loads(l); print(d['mode'], 'multi' if d['multi'] else 'single', d['rep'], d['records'], d.get('walk_mmap_register_ms'), d['replay_ms'], d.get('unregister_unmap_ms'), d['open_ms'])
"
