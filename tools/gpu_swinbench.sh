#!/bin/bash
# SwinUNETR (config c4) bench + rocprofv3 kernel stats.  usage: bash tools/gpu_swinbench.sh TAG [PROF]
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=${1:-sb}
O=$R/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python3 $R/bench.py --model swin_unetr --size 128 --batch 1 --steps 5 --warmup 2 --timer-steps 1 > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-600
if [ -n "$2" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o prof -- python3 $R/bench.py --model swin_unetr --size 128 --batch 1 --steps 3 --warmup 1 --timer-steps 0 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
  python3 $R/tools/rocprof_families.py stats $O/trace/prof_kernel_stats.csv 4 > $O/families.txt; head -40 $O/families.txt
fi
