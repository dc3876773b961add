#!/bin/bash
# r06c: wgrad_row tuning A/B (MMSEG_WGRAD_ROW_V: 0 = 4 rows / 4 slots, 1 = 5 slots, 2 = prio for waves 6..11,
# 3 = 6 rows per step), convbench at 96^3 and the c3 step
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06c
mkdir -p $O
cd $R
for V in 0 1 2 3 0; do
  MMSEG_WGRAD_ROW_V=$V timeout -k 10 300 python3 tools/convbench.py --shape 2,96,32,32 2,96,64,32 --only wgrad,wgradn --iters 40 > $O/cb_v$V.log 2>&1 || { tail -5 $O/cb_v$V.log; exit 1; }
  echo "V=$V $(grep -v amdgpu.ids $O/cb_v$V.log | python3 -c "import sys,json; print(' '.join(f\"{d['shape']}/{d['op']}:{d['us']}\" for d in map(json.loads, sys.stdin)))")"
done
for V in 0 3 1 0 3 1; do
  MMSEG_WGRAD_ROW_V=$V timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_v$V.log 2>&1 || { tail -5 $O/bench_v$V.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/bench_v$V.log').read().strip().split('\n')[-1])
f=d['kernel_families']; print('V=$V', d['ms_per_step'], {k: v['ms_per_step'] for k, v in f.items() if 'wgrad_row' in k})"
done
echo r06c done
