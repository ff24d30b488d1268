set -e
for rep in 1 2; do
  for v in "--fused" "--fused --chunk-kib 256" "--fused --chunk-kib 1024" ""; do
    timeout -k 10 200 python bench.py $v --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/xc.json 2>/dev/null
    echo "[$v] $(python3 -c "import json; d=json.loads(open('gpurun_out/xc.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], {k: round(v,3) for k,v in d['phase_ms'].items()})")"
  done
done
