set -o pipefail
out=gpurun_out/r4t
mkdir -p $out
GCK_LIB_PATH=gocask_amd/var/libgocask_hip_full_time.so timeout -k 10 200 python tools/scrub_time.py > $out/scrub_time.json 2> $out/scrub_time.err || { tail $out/scrub_time.err; exit 1; }
cat $out/scrub_time.json
