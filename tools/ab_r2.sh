# Interleaved step-time A/B of a second tree (default abr2/: the round-2 head
# f864365, git archive + make) against the working tree on one box, then the
# in-kernel clock of k_crc_rows and of the stream read (stamps build):
#   bash tools/ab_r2.sh [other-tree] [reps] > gpurun_out/<tag>/ab.log
set -o pipefail
other=${1:-abr2}; reps=${2:-3}
for rep in $(seq $reps); do
  for t in "$other" .; do
    ( cd $t && timeout -k 10 150 python bench.py --no-cpu-baseline --steps 20 --warmup 3 2>/dev/null | python3 -c "
import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d['roofline']
print('$t', 'step', d['ms_per_step'], 'crc_rows', round(r['crc_rows_ms'],3), 'stream_gbs', r['stream_read_gbs'],
      'stream_ms', round(34359738368/r['stream_read_gbs']/1e6, 3), {k: round(v,3) for k,v in d['phase_ms'].items()})" ) || exit 1
  done
done
if [ -f gocask_amd/var/libgocask_hip_clk.so ]; then
  for rep in 1 2; do
    GCK_LIB_PATH=gocask_amd/var/libgocask_hip_clk.so timeout -k 10 150 python tools/clock.py || exit 1
  done
fi
