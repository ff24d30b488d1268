#!/bin/bash
# Pipeline shape A/B on one box (GCK_PIPE="groups,first_group_permille"),
# interleaved, REPS rounds:  bash tools/xp_pipe.sh "1,500" "4,250" ...
set -o pipefail
for rep in ${REPS:-1 2}; do
for shape in "$@"; do
  printf "%s rep %s: " "$shape" "$rep"
  GCK_PIPE=$shape timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 --warmup 3 ${BENCH_ARGS:-} | python3 -c "
import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1])
print(d['ms_per_step'], d['value'], {k: round(v,3) for k,v in d['phase_ms'].items()})" || exit 1
done
done
