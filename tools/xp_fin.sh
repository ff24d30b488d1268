# Finalize beside the CRC pass: shapes (GCK_FSPLIT, permille of the rows per
# piece; "0" = no cut) and side-CU masks (GCK_FMASK) on C3, interleaved
#   bash tools/xp_fin.sh ["cfg1" "cfg2" ...]
set -e
cfgs=("$@")
[ ${#cfgs[@]} -eq 0 ] && cfgs=("GCK_FSPLIT=0" "GCK_FSPLIT=450,300,170,80" "GCK_FMASK=2" "GCK_FSPLIT=500,300,200" "GCK_FSPLIT=350,250,180,130,90")
for rep in ${REPS:-1 2}; do
for cfg in "${cfgs[@]}"; do
  echo "CFG=$cfg"
  env $cfg timeout -k 10 120 python bench.py --no-cpu-baseline --steps 5 --warmup 2 --verbose | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'], d['config'].get('crc_rejects'), {k: round(v,3) for k,v in d['phase_ms'].items()})"
done
done
