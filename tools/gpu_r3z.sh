set -o pipefail
out=gpurun_out/r3z
mkdir -p $out
export TMPDIR=/tmp
for mib in 8 32; do
GCK_STAGE_MIB=$mib SHIM_THREADS="8 16" GCK_REPLAY_TRACE=1 timeout -k 10 600 python tools/shim_c3.py 2 1 > $out/shim_$mib.jsonl 2> $out/shim_$mib.err || { tail -20 $out/shim_$mib.err; exit 1; }
python3 -c "
import json
for l in open('$out/shim_$mib.jsonl'):
    d=json.loads(l); print('$mib MiB', d['mode'], d['copy_threads'], d['rep'], d['replay_ms'], d['open_ms']); print('\n'.join(d.get('trace',[])[:1]+d.get('trace',[])[-2:]))
"
done
