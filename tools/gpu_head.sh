#!/bin/bash
# fused head + loss variants (tools/headbench.py, one process per setting: the chunkings are read once)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-head}
mkdir -p $O
hb() { timeout -k 10 120 env "$@" python3 $R/tools/headbench.py --step-only --iters 30 >> $O/hb.log 2>&1 || { tail -20 $O/hb.log; exit 1; }; tail -1 $O/hb.log; }
hb MMSEG_X=0
hb MMSEG_HEAD_PF=1
hb MMSEG_LOSS_VPC=1728
hb MMSEG_LOSS_VPC=1728 MMSEG_HEAD_PF=1
hb MMSEG_LOSS_VPC=1024 MMSEG_HEAD_PF=1
hb MMSEG_HEAD_BWD_VPC=3456
hb MMSEG_HEAD_BWD_VPC=1024
hb MMSEG_LOSS_VPC=3456 MMSEG_HEAD_PF=1
hb MMSEG_X=1
