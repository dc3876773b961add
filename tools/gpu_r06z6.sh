#!/bin/bash
# r06z6: c4 profile set (trace + PMC passes + judged line) of the fused AdamW + pack / head-backward tree
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash $R/tools/gpu_profile.sh r06z6 c4 --model swin_unetr --size 128 --batch 1 || exit 1
echo r06z6 done
