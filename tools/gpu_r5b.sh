set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r5b
mkdir -p $out
bash tools/ktrace.sh r5b > $out/kt.log 2>&1 || { tail -20 $out/kt.log; exit 1; }
python3 tools/timeline.py gpurun_out/kt_r5b > $out/timeline.json || exit 1
cat $out/timeline.json
L=gocask_amd/var
bash tools/ab_mix.sh 3 gocask_amd/libgocask_hip.so $L/libgocask_hip_st8.so $L/libgocask_hip_st6.so $L/libgocask_hip_st2.so $L/libgocask_hip_eb.so > $out/ab.log 2>&1 || { cat $out/ab.log; exit 1; }
cut -c1-260 $out/ab.log
