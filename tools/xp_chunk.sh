# Boundary-phase sensitivity to the speculation chunk size (bench --chunk-kib).
set -e
for ck in 128 256 512 1024 2048; do
  echo "CHUNK=$ck"
  timeout -k 10 120 python bench.py --no-cpu-baseline --steps 5 --warmup 2 --chunk-kib $ck --verbose | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'], d.get('fixups'), d.get('overflow_chunks'), {k: round(v,3) for k,v in d['phase_ms'].items()})"
done
