# C3 Open by path (shim) with several library builds, interleaved:
#   bash tools/shim_ab.sh dir1 dir2 ...   (each dir holds a libgocask_hip.so)
set -o pipefail
out=gpurun_out/shim_ab
mkdir -p $out
: > $out/ab.jsonl
for d in "$@"; do echo "$d" >> $out/dirs; done
SHIM_AB_DIRS="$*" GCK_REPLAY_TRACE=1 timeout -k 10 900 python tools/shim_c3.py 2 1 > $out/ab.jsonl 2> $out/ab.err || { tail -20 $out/ab.err; exit 1; }
python3 -c "
import json
for l in open('$out/ab.jsonl'):
    d=json.loads(l); print(d.get('libdir'), d['mode'], d['rep'], d['replay_ms'], d['open_ms'], [t for t in d.get('trace',[]) if 'ready' in t or 'results' in t])
"
