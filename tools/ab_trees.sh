# Interleaved step-time A/B of several built trees on one box (C3, bench.py):
#   bash tools/ab_trees.sh <reps> <tree1> <tree2> ...   -> one line per run
set -o pipefail
reps=$1; shift
for rep in $(seq $reps); do
  for t in "$@"; do
    ( cd $t && timeout -k 10 150 python bench.py --no-cpu-baseline --steps 20 --warmup 3 2>/dev/null | python3 -c "
import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d['roofline']
print('$t', 'step', d['ms_per_step'], 'crc_rows', round(r['crc_rows_ms'],3), 'stream_ms', round(34359738368/r['stream_read_gbs']/1e6, 3),
      {k: round(v,3) for k,v in d['phase_ms'].items()})" ) || exit 1
  done
done
