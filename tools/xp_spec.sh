# Boundary-phase sweep over the speculation chunk, window and stage capacity
# (bench --chunk-kib / --spec-kib / --chunk-cap):
#   bash tools/xp_spec.sh "128:4:4096 64:4 ..."
set -e
for cw in ${1:-64:4 128:4 128:8 256:4 256:8 512:512}; do
  IFS=: read ck sw cap <<< "$cw"; cap=${cap:-0}
  echo "CHUNK=$ck WINDOW=$sw CAP=$cap: $(timeout -k 10 120 python bench.py --no-cpu-baseline --steps 5 --warmup 2 --chunk-kib $ck --spec-kib $sw --chunk-cap $cap --verbose 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'], 'fix', d.get('fixups'), 'ovf', d.get('overflow_chunks'), {k: round(v,3) for k,v in d['phase_ms'].items()})")"
done
