#!/bin/bash
# r06h: window-attention microbench at c4 shapes; qb2 with and without per-window restaging (timing experiment)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06h
mkdir -p $O
cd $R
timeout -k 10 120 python3 tools/wabench.py --stages 0,1,2,3 > $O/wa0.log 2>&1 || { tail -20 $O/wa0.log; exit 1; }
cat $O/wa0.log
MMSEG_WA_EXP=1 timeout -k 10 120 python3 tools/wabench.py --stages 0,1 > $O/wa1.log 2>&1 || { tail -20 $O/wa1.log; exit 1; }
cat $O/wa1.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof -o wa -- python3 $R/tools/wabench.py --stages 0,1,2,3 --reps 10 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" | head -3
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); head -12 "$f"
echo r06h done
