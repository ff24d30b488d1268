# Default vs fused run path on one box (bench ms/step, interleaved), then the
# fused kernel with and without its parse under rocprof:
#   bash tools/xp_paths.sh
set -e
export TMPDIR=/tmp
for rep in ${PREPS:-1 2}; do
  for mode in default fused; do
    flag=""; [ $mode = fused ] && flag="--fused"
    timeout -k 10 200 python bench.py $flag --no-cpu-baseline --steps 10 --warmup 3 --verbose > gpurun_out/path_${mode}_$rep.json 2>gpurun_out/path_${mode}_$rep.err
    echo "$mode $rep: $(python3 -c "import json; d=json.loads(open('gpurun_out/path_${mode}_$rep.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], {k: round(v,3) for k,v in d['phase_ms'].items()})")"
  done
done
[ -n "$NOFAB" ] || bash tools/xp_fused_ab.sh uni=gocask_amd/libgocask_hip.so noparse=gocask_amd/var/libgocask_hip_noparse.so
