#!/bin/bash
# r06x2: final round-6 build -- c2, c4, c5 profile sets (trace + PMC passes + judged line each)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash $R/tools/gpu_profile.sh r06x c2 --model unet || exit 1
bash $R/tools/gpu_profile.sh r06x c4 --model swin_unetr --size 128 --batch 1 || exit 1
bash $R/tools/gpu_profile.sh r06x c5 --modalities CT,PET,MRI --loss tversky || exit 1
echo r06x2 done
