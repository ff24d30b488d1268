# A/B of fused-path builds (bench --fused): tools/xp_fused.sh lib1.so lib2.so ...
set -e
for lib in "$@"; do
  echo "LIB=$lib"
  GCK_LIB_PATH=$lib timeout -k 10 120 python bench.py --fused --no-cpu-baseline --steps 5 --warmup 2 --verbose | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'], {k: round(v,3) for k,v in d['phase_ms'].items()})"
done
