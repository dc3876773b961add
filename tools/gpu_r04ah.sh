#!/bin/bash
# runtime-brick weight-gradient split knobs on the grouped tree: c3 A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
AB_STEPS=40 bash $R/tools/gpu_ab.sh r04ah_ab - MMSEG_WGRAD_RSLOTS=384 MMSEG_WGRAD_RSLOTS=512 MMSEG_WGRAD_RMINB=2 MMSEG_WGRAD_RMINB=8 - MMSEG_WGRAD_RSLOTS=384 MMSEG_WGRAD_RSLOTS=512 MMSEG_WGRAD_RMINB=2 MMSEG_WGRAD_RMINB=8
