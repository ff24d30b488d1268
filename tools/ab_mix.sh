# Interleaved step-time A/B on one box (C3, bench.py): each argument is a built
# tree (its own bench.py and library) or a library of this tree (GCK_LIB_PATH).
#   bash tools/ab_mix.sh <reps> <tree-or-lib> ...   -> one line per run
set -o pipefail
reps=$1; shift
for rep in $(seq $reps); do
  for t in "$@"; do
    if [ -d "$t" ]; then dir=$t; lib=; else dir=.; lib=$t; fi
    diag=; [ -n "$lib" ] && [ -f "${lib/libgocask_hip/libgocask_diag}" ] && diag=${lib/libgocask_hip/libgocask_diag}
    ( cd $dir && GCK_LIB_PATH=$lib GCK_DIAG_PATH=$diag timeout -k 10 150 python bench.py --no-cpu-baseline --steps 20 --warmup 3 2>/dev/null | python3 -c "
import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d['roofline']
print('$t', 'step', d['ms_per_step'], 'crc_rows', round(r['crc_rows_ms'],3), 'stream_ms', round(34359738368/r['stream_read_gbs']/1e6, 3),
      {k: round(v,3) for k,v in d['phase_ms'].items()})" ) || exit 1
  done
done
