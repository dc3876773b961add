#!/bin/bash
# r06g: per-launch timer dump of the c3 step (issue order: which IN passes remain where) and the c4 bench line
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06g
mkdir -p $O
cd $R
timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --timer-steps 1 --timer-dump $O/c3_launches.json --no-cpu-baseline > $O/bench_c3.log 2>&1 || { tail -20 $O/bench_c3.log; exit 1; }
tail -c 300 $O/bench_c3.log
timeout -k 10 400 python3 bench.py --model swin_unetr --steps 10 --warmup 3 --timer-steps 1 --timer-dump $O/c4_launches.json --no-cpu-baseline > $O/bench_c4.log 2>&1 || { tail -20 $O/bench_c4.log; exit 1; }
tail -c 300 $O/bench_c4.log
echo r06g done
