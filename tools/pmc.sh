#!/bin/bash
# Profiling passes on the bench command (run on the GPU box from the repo root):
#   1. kernel trace + stats (per-kernel average durations)
#   2..n. PMC counters, one pass each (never combined with runtime/sys traces)
# Usage: tools/pmc.sh <tag> [bench args...]   -> gpurun_out/prof_<tag>/
#   PMC_EXTRA="..." adds bench flags to the counter passes
set -o pipefail
tag=${1:-r1}; shift
args=${*:---steps 5 --warmup 2 --no-cpu-baseline --keydir --merge}
export TMPDIR=/tmp
out=gpurun_out/prof_$tag
mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- \
  python3 bench.py $args > $out/trace.log 2>&1 || exit $?
i=0
for ctrs in "FETCH_SIZE" "WRITE_SIZE" \
    "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
    "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VMEM" \
    "TCC_HIT_sum TCC_MISS_sum TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE" \
    "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $ctrs --kernel-include-regex "k_crc_rows|k_stream_read|k_spec_entry|k_walk|k_finalize|k_row_plan|k_compact|k_row_index|k_kd_insert|k_key_hash|k_verify|k_mg_insert" \
    --output-format csv -d $out/pmc$i -o run -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline --keydir $PMC_EXTRA \
    > $out/pmc$i.log 2>&1 || exit $?
done
