set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r4h
mkdir -p $out
bash tools/ab_mix.sh 3 . gocask_amd/var/libgocask_hip_claim1.so gocask_amd/var/libgocask_hip_static6.so gocask_amd/var/libgocask_hip_c1s6.so > $out/ab_queue.log 2>&1
rc=$?
cat $out/ab_queue.log
[ $rc -ne 0 ] && exit $rc
i=0
for ctrs in "SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_LEVEL_VMEM SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" \
    "TA_BUSY_avr TA_BUSY_max TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum GRBM_GUI_ACTIVE" \
    "TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TD_TD_BUSY_sum"; do
  i=$((i+1))
  timeout -k 10 -s KILL 120 rocprofv3 --pmc $ctrs --kernel-include-regex "k_finalize|k_walk|k_spec_entry|k_crc_rows|k_compact" \
    --output-format csv -d $out/pmc$i -o run -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline > $out/pmc$i.log 2>&1 || exit $?
done
echo pmc done
