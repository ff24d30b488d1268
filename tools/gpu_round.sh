#!/bin/bash
# One GPU call that re-measures a build end to end (run from the repo root on
# the GPU box, replaces the per-experiment launchers of rounds 3-4):
#   bash tools/gpu_round.sh <tag> [steps...]      -> gpurun_out/<tag>/
# steps (default: suite smoke bench pmc): suite | smoke | bench | pmc | kt |
#   secondary (encoder, scrub, Get, compaction) | clock | ab:<lib1>,<lib2>,...
set -o pipefail
tag=${1:?tag}; shift
steps=${*:-suite smoke bench pmc}
export TMPDIR=/tmp
out=gpurun_out/$tag
mkdir -p $out
for s in $steps; do
  case $s in
  suite)
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $out/gpu_suite.log 2>&1 \
      || { tail -30 $out/gpu_suite.log; exit 1; }
    tail -1 $out/gpu_suite.log ;;
  smoke)
    timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { cat $out/smoke.log; exit 1; }
    tail -1 $out/smoke.log ;;
  bench)
    timeout -k 10 300 python bench.py > $out/bench_default.json 2> $out/bench_default.err || { tail -20 $out/bench_default.err; exit 1; }
    cut -c1-900 $out/bench_default.json ;;
  pmc)
    bash tools/pmc.sh $tag || exit $? ;;
  kt)
    bash tools/ktrace.sh $tag || exit $? ;;
  clock)
    # the stamps build (tools/clock.py's header: make ... EXTRA=-DGCK_CLOCK_STAMPS)
    GCK_LIB_PATH=gocask_amd/var/libgocask_hip_clk.so timeout -k 10 150 python tools/clock.py > $out/clock.log 2>&1 \
      || { cat $out/clock.log; exit 1; }
    cat $out/clock.log ;;
  secondary)
    for rep in 1 2 3; do timeout -k 10 120 python tools/bench_encode.py 2>/dev/null | tail -1 >> $out/bench_encode.log || exit 1; done
    for rep in 1 2 3; do timeout -k 10 150 python tools/scrub.py 2>/dev/null | tail -1 >> $out/scrub.log || exit 1; done
    for rep in 1 2; do timeout -k 10 300 python tools/bench_get.py 2>/dev/null | tail -1 >> $out/bench_get.log || exit 1; done
    for rep in 1 2; do timeout -k 10 300 python tools/bench_compact.py 2>/dev/null | tail -1 >> $out/bench_compact.log || exit 1; done
    cut -c1-200 $out/bench_encode.log $out/scrub.log $out/bench_get.log $out/bench_compact.log ;;
  ab:*)
    bash tools/ab_mix.sh 3 $(echo ${s#ab:} | tr , ' ') > $out/ab.log 2>&1 || { cat $out/ab.log; exit 1; }
    cut -c1-300 $out/ab.log ;;
  *) echo "unknown step $s"; exit 2 ;;
  esac
done
