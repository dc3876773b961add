#!/bin/bash
# r06i: token-linear GEMM A/B (64x192 / 128x48 point tiles vs the previous build), then the new build's c4 line
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06i
mkdir -p $O
cd $R
timeout -k 10 200 python3 tools/pointbench.py --lib $R/tools/_ab/libmmseg_hip_old.so > $O/pb_old.log 2>&1 || { tail -20 $O/pb_old.log; exit 1; }
timeout -k 10 200 python3 tools/pointbench.py > $O/pb_new.log 2>&1 || { tail -20 $O/pb_new.log; exit 1; }
cat $O/pb_old.log $O/pb_new.log
true
: "
import json; d=json.loads(open('$O/bench_c4.log').read().strip().split('\n')[-1]); print(d['ms_per_step'], d['value'])
f=d['kernel_families']
for k,v in sorted(f.items(), key=lambda kv:-kv[1]['ms_per_step'])[:14]: print(k, v['ms_per_step'])"
echo r06i done
