# Scrub and encoder A/B of the working tree against a second tree (built in
# place), interleaved on one box:  bash tools/ab_tree_sec.sh <other-tree> [reps]
set -o pipefail
other=$1; reps=${2:-2}
for rep in $(seq $reps); do
  for t in "$other" .; do
    echo "$t scrub $( cd $t && timeout -k 10 150 python tools/scrub.py 2>/dev/null | tail -1 )" || exit 1
    echo "$t encode $( cd $t && timeout -k 10 120 python tools/bench_encode.py --gib 1 2>/dev/null | tail -1 )" || exit 1
  done
done
