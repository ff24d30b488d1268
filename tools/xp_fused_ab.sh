# A/B of fused-path builds by rocprof kernel time (k_fuse full launches):
#   bash tools/xp_fused_ab.sh tag1=lib1.so tag2=lib2.so ...
set -e
export TMPDIR=/tmp
for rep in ${REPS:-1 2}; do
for tl in "$@"; do
  tag=${tl%%=*}; lib=${tl#*=}
  GCK_LIB_PATH=$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/fab_${tag}_$rep -o run -- python bench.py --fused --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/fab_${tag}_$rep.log 2>&1
  echo "$tag rep $rep ok"
done
done
