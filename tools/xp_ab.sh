# A/B two builds of the library on the same box (box-to-box variance is large).
set -e
for lib in gocask_amd/libgocask_hip.so gocask_amd/var/libgocask_hip_plan.so gocask_amd/libgocask_hip.so gocask_amd/var/libgocask_hip_plan.so; do
  echo "LIB=$lib"
  GCK_X_MODE=2 GCK_LIB_PATH=$lib timeout -k 10 120 python bench.py --no-cpu-baseline --steps 5 --warmup 2 | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'], {k: round(v,3) for k,v in d['phase_ms'].items()})"
done
