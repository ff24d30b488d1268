set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r5a
mkdir -p $out
timeout -k 10 300 python bench.py --no-cpu-baseline > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
cut -c1-1200 $out/bench.json
timeout -k 10 300 python tools/ceiling.py > $out/ceiling.json 2> $out/ceiling.err || { tail -20 $out/ceiling.err; exit 1; }
cat $out/ceiling.json
GCK_LIB_PATH=gocask_amd/var/libgocask_hip_clk.so timeout -k 10 300 python tools/ceiling.py --reps 1 > $out/ceiling_clk.json 2> $out/ceiling_clk.err || { tail -20 $out/ceiling_clk.err; exit 1; }
cat $out/ceiling_clk.json
