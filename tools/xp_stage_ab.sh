# A/B of the staging allocation (registered huge pages vs hipHostMalloc) on
# the C3 live Open by path, modes interleaved in one box
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r6p
SHIM_MODES="5 6" GCK_REPLAY_TRACE=1 timeout -k 10 600 python tools/shim_c3.py ${REPS:-4} > gpurun_out/r6p/ab_stage.jsonl 2>/dev/null || exit 1
python3 -c "
import json
for l in open('gpurun_out/r6p/ab_stage.jsonl'):
    d=json.loads(l); t=d['trace']; print('hm' if d['stage_hostmalloc'] else 'reg', d['rep'], d['replay_ms'], d['open_ms'], t[0][14:120], [x for x in t if 'groups' in x][0][14:])
"
