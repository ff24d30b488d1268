# C4 (one rank's 16 x 2 GiB shard) kernel trace + FETCH/WRITE passes -> profiles/traffic_c4.json
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/prof_r4l
mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- \
  python3 bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline > $out/trace.log 2>&1 || exit $?
i=0
for ctrs in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 -s KILL 300 rocprofv3 --pmc $ctrs --kernel-include-regex "k_crc_rows|k_stream_read" \
    --output-format csv -d $out/pmc$i -o run -- python3 bench.py --config c4 --steps 2 --warmup 0 --no-cpu-baseline \
    > $out/pmc$i.log 2>&1 || exit $?
done
tail -1 $out/trace.log
