#!/bin/bash
# r06z4: the tree after the fused AdamW + pack and the head backward -- whole GPU suite + smoke, then the c3 profile
# set (trace + PMC passes + judged line)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash $R/tools/gpu_check.sh r06z4 || exit 1
bash $R/tools/gpu_profile.sh r06z4 c3 || exit 1
echo r06z4 done
