set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r6n
SHIM_MODES="5" GCK_REPLAY_TRACE=1 timeout -k 10 600 python tools/shim_c3.py ${REPS:-3} > gpurun_out/r6n/shim_live.jsonl 2> gpurun_out/r6n/shim_live.err
rc=$?
tail -60 gpurun_out/r6n/shim_live.err
cut -c1-600 gpurun_out/r6n/shim_live.jsonl
exit $rc
