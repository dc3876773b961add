#!/bin/bash
# r06z8: c3 (headline) profile set and judged line re-taken on a second box (the r06z4 box ran every MFMA family
# 7-9 % slower than the r06x / r06z boxes at equal HBM-pass times)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash $R/tools/gpu_profile.sh r06z8 c3 || exit 1
echo r06z8 done
