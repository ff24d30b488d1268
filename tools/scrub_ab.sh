# A/B builds of the keydir scrub (tools/scrub.py), each twice, interleaved
set -e
for rep in 1 2; do for lib in "$@"; do
  echo "$lib $(GCK_LIB_PATH=$lib timeout -k 10 150 python tools/scrub.py 2>/dev/null | tail -1)"
done; done
