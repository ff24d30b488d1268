# Round 4 call d: bisect the k_crc_rows regression over round-3 commits (one box, interleaved)
set -o pipefail
mkdir -p gpurun_out/r4d
bash tools/ab_trees.sh 2 abr2 bis/42d18c0 bis/55f6d80 bis/063e4bf bis/34bbb6c bis/e65c234 . > gpurun_out/r4d/bisect.log 2>&1
rc=$?
cat gpurun_out/r4d/bisect.log
exit $rc
