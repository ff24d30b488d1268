# A/B builds of the library on one box (box-to-box variance is large):
#   bash tools/xp_ab.sh lib1.so lib2.so ...   (each run twice, interleaved)
set -e
for rep in ${REPS:-1 2}; do
for lib in "$@"; do
  echo "LIB=$lib"
  GCK_LIB_PATH=$lib timeout -k 10 120 python bench.py --no-cpu-baseline --steps 5 --warmup 2 --verbose | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'], d.get('fixups'), {k: round(v,3) for k,v in d['phase_ms'].items()})"
done
done
