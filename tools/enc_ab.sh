# A/B builds of the encoder (tools/bench_encode.py), each twice, interleaved
for rep in 1 2; do for lib in "$@"; do
  echo "$lib $(GCK_LIB_PATH=$lib timeout -k 10 120 python tools/bench_encode.py 2>/dev/null | tail -1)"
done; done
