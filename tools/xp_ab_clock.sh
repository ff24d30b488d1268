set -o pipefail
TAG=${1:?tag}
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
bash tools/ab_mix.sh 3 gocask_amd/var/libgocask_hip_base.so gocask_amd/libgocask_hip.so > gpurun_out/$TAG/ab.log 2>&1 || { cat gpurun_out/$TAG/ab.log; exit 1; }
cat gpurun_out/$TAG/ab.log
GCK_LIB_PATH=gocask_amd/var/libgocask_hip_clk.so timeout -k 10 150 python tools/phase_clock.py > gpurun_out/$TAG/phase_clock.json 2> gpurun_out/$TAG/phase_clock.err || { tail -20 gpurun_out/$TAG/phase_clock.err; exit 1; }
cat gpurun_out/$TAG/phase_clock.json
