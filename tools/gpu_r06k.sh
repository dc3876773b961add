#!/bin/bash
# r06k: rocprofv3 trace + PMC passes + judged bench line for c3 and c4 on the round-6 build
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash $R/tools/gpu_profile.sh r06k c3 || exit 1
bash $R/tools/gpu_profile.sh r06k c4 --model swin_unetr --size 128 --batch 1 || exit 1
echo r06k done
