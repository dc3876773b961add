#!/bin/bash
# 32-co weight-gradient row tiles at small volumes (half the split partials): c3 A/B on the grouped tree
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
AB_STEPS=40 bash $R/tools/gpu_ab.sh r04u_ab - MMSEG_WGRAD_RCO64_MINV=10000 MMSEG_WGRAD_RCO64_MINV=100000 MMSEG_WGRAD_CO64_MINV=100000 - MMSEG_WGRAD_RCO64_MINV=10000 MMSEG_WGRAD_RCO64_MINV=100000 MMSEG_WGRAD_CO64_MINV=100000
