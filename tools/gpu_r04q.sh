#!/bin/bash
# runtime-brick chunk split: whole-step A/B (c3, c5) of the no-split threshold / slot count
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
AB_STEPS=40 bash $R/tools/gpu_ab.sh r04q_ab - MMSEG_BRICKR_NOSPLIT=192 MMSEG_BRICKR_SLOTS=128 - MMSEG_BRICKR_NOSPLIT=192 MMSEG_BRICKR_SLOTS=128 || exit 1
AB_STEPS=30 bash $R/tools/gpu_ab.sh r04q_c5 "--modalities CT,PET,MRI --loss tversky" "MMSEG_BRICKR_NOSPLIT=192 --modalities CT,PET,MRI --loss tversky" "--model unet" "MMSEG_BRICKR_NOSPLIT=192 --model unet"
