#!/bin/bash
# rocprofv3 kernel trace of the c4 SwinUNETR bench (128^3 fs48 B=1).  usage: bash tools/gpu_c4prof.sh TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-c4prof}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o prof -- python3 $R/bench.py --model swin_unetr --size 128 --batch 1 --steps 4 --warmup 2 --timer-steps 0 --no-cpu-baseline > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
tail -1 $O/prof.log | cut -c1-200
python3 $R/tools/rocprof_families.py stats $O/trace/prof_kernel_stats.csv 6 > $O/families.txt 2>&1; head -45 $O/families.txt
python3 $R/tools/rocprof_families.py steady $O/trace/prof_kernel_trace.csv $O/steady.json 2 > $O/families_steady.txt 2>&1; head -40 $O/families_steady.txt
