#!/bin/bash
# r06l: token-linear microbench with the 64x128 point tile; c4 bench line
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06l
mkdir -p $O
cd $R
timeout -k 10 200 python3 tools/pointbench.py > $O/pb.log 2>&1 || { tail -20 $O/pb.log; exit 1; }
cat $O/pb.log
timeout -k 10 600 python3 bench.py --model swin_unetr --size 128 --batch 1 --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_c4.log 2>&1 || { tail -20 $O/bench_c4.log; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench_c4.log').read().strip().split('\n')[-1]); print(d['ms_per_step'], d['value'])
f=d['kernel_families']
for k,v in sorted(f.items(), key=lambda kv:-kv[1]['ms_per_step'])[:16]: print(k, v['ms_per_step'])"
echo r06l done
