#!/bin/bash
# fused head + loss chunk sizes after the bf16-MFMA change: headbench over MMSEG_LOSS_VPC / MMSEG_HEAD_BWD_VPC, then c3 A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04ag
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in "MMSEG_LOSS_VPC=1728" "MMSEG_LOSS_VPC=864" "MMSEG_LOSS_VPC=1152" "MMSEG_LOSS_VPC=3456" "MMSEG_HEAD_BWD_VPC=3456" "MMSEG_HEAD_BWD_VPC=1728" "MMSEG_HEAD_BWD_VPC=2592" "MMSEG_HEAD_BWD_VPC=6912"; do
  env $v timeout -k 10 120 python3 $R/tools/headbench.py --step-only > $O/hb.log 2>&1 || { tail -20 $O/hb.log; exit 1; }
  echo "== $v $(tail -1 $O/hb.log)"
done
