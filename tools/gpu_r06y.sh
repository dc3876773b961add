#!/bin/bash
# r06y: final tree after the window-attention pipeline -- whole GPU suite + smoke, then the c4 profile set
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash $R/tools/gpu_check.sh r06y || exit 1
bash $R/tools/gpu_profile.sh r06y c4 --model swin_unetr --size 128 --batch 1 || exit 1
echo r06y done
