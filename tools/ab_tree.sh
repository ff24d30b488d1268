# Step-time A/B of the working tree against a second tree (e.g. ab/head from
# git archive HEAD, built in place), interleaved on one box:
#   bash tools/ab_tree.sh <other-tree> [reps]   -> one line per run
set -o pipefail
other=$1; reps=${2:-3}
for rep in $(seq $reps); do
  for t in "$other" .; do
    ( cd $t && timeout -k 10 150 python bench.py --no-cpu-baseline --steps 10 --warmup 3 2>/dev/null | python3 -c "
import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1])
print('$t', d['ms_per_step'], round(d['roofline']['crc_rows_ms'],3), {k: round(v,3) for k,v in d['phase_ms'].items()})" ) || exit 1
  done
done
