set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r5c
mkdir -p $out
L=gocask_amd/var
bash tools/ab_mix.sh 3 $L/libgocask_hip_base.so gocask_amd/libgocask_hip.so $L/libgocask_hip_st8.so $L/libgocask_hip_eb.so $L/libgocask_hip_gtab.so > $out/ab.log 2>&1 || { cat $out/ab.log; exit 1; }
cut -c1-260 $out/ab.log
GCK_LIB_PATH=gocask_amd/var/libgocask_hip_clk.so timeout -k 10 200 python tools/phase_clock.py > $out/phase_clock.json 2> $out/phase_clock.err || { tail -20 $out/phase_clock.err; exit 1; }
cat $out/phase_clock.json
