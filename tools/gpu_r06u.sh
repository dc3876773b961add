#!/bin/bash
# r06u: c4 whole-step A/B of the runtime-brick slot target (MMSEG_BRICKR_SLOTS 256 default / 512 / 1024)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06u
mkdir -p $O
cd $R
for v in 256 512 1024 256 512 1024; do
  MMSEG_BRICKR_SLOTS=$v timeout -k 10 400 python3 bench.py --model swin_unetr --size 128 --batch 1 --steps 10 --warmup 3 --no-cpu-baseline > $O/c4_$v.log 2>&1 || { tail -20 $O/c4_$v.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/c4_$v.log').read().strip().split('\n')[-1]); f=d['kernel_families']
print('SLOTS=$v', d['ms_per_step'], {k: f[k]['ms_per_step'] for k in f if 'brickr' in k or 'splitk' in k})"
done
