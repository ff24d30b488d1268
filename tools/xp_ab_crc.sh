# A/B of library builds on one box, interleaved: bench step + k_crc_rows
# ablation (mode 0 = as shipped, mode 8 = synthetic bytes: compute only).
#   bash tools/xp_ab_crc.sh lib1.so lib2.so ...
set -e
for rep in ${REPS:-1 2 3}; do
for lib in "$@"; do
  echo "LIB=$lib"
  GCK_LIB_PATH=$lib timeout -k 10 120 python bench.py --no-cpu-baseline --steps 10 --warmup 3 --verbose | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'], {k: round(v,3) for k,v in d['phase_ms'].items()})"
  GCK_LIB_PATH=$lib timeout -k 10 120 python tools/ablate.py c3 0,8 | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print({k: v for k,v in d.items() if k.startswith('mode') and k.endswith('_ms') or k=='stream'})"
done
done
