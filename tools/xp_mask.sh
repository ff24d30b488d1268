set -e
for rep in 1 2; do
for cfg in "" "GCK_XP_MASK=1" "GCK_XP_MASK=2" "GCK_XP_MASK=3" "GCK_XP_MASK=2 GCK_XP_FINSIDE=1" "GCK_XP_MASK=3 GCK_XP_FINSIDE=1"; do
  echo "CFG=$cfg"
  env $cfg GCK_LIB_PATH=gocask_amd/var/libgocask_hip_mask.so timeout -k 10 120 python bench.py --no-cpu-baseline --steps 5 --warmup 2 --verbose | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'], d['config'].get('crc_rejects'), {k: round(v,3) for k,v in d['phase_ms'].items()})"
done
done
