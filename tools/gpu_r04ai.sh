#!/bin/bash
# runtime-brick column-tile / slot knobs on the final tree: c3 A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
AB_STEPS=40 bash $R/tools/gpu_ab.sh r04ai_ab - MMSEG_BRICKR_BN32_BLK=512 MMSEG_BRICKR_SLOTS=128 MMSEG_BRICKR_SLOTS=384 - MMSEG_BRICKR_BN32_BLK=512 MMSEG_BRICKR_SLOTS=128 MMSEG_BRICKR_SLOTS=384
