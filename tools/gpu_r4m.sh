set -o pipefail
out=gpurun_out/r4m
mkdir -p $out
timeout -k 10 300 python tools/chase_win.py > $out/chase_win.json 2> $out/chase_win.err || { tail -20 $out/chase_win.err; exit 1; }
cat $out/chase_win.json
timeout -k 10 300 python tools/chase.py > $out/chase.json 2> $out/chase.err || { tail -20 $out/chase.err; exit 1; }
cat $out/chase.json
