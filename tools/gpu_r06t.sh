#!/bin/bash
# r06t: c3 whole-step A/B of the 24^3 grouping mode (MMSEG_GROUP_FORCE_R=1 default: grouped runtime-brick launches;
# 0: per-modality brick2 / wgrad_dma launches at 24^3), interleaved on one box
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06t
mkdir -p $O
cd $R
for v in 1 0 1 0 1 0; do
  MMSEG_GROUP_FORCE_R=$v timeout -k 10 300 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline > $O/c3_$v.log 2>&1 || { tail -20 $O/c3_$v.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/c3_$v.log').read().strip().split('\n')[-1]); print('FORCE_R=$v', d['ms_per_step'])"
done
