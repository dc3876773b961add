#!/bin/bash
# r06zd: c4 profile set (trace + PMC passes + judged line) of the final tree (head data gradient on 2,048 blocks)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash $R/tools/gpu_profile.sh r06zd c4 --model swin_unetr --size 128 --batch 1 || exit 1
echo r06zd done
