#!/bin/bash
# r06x1: final round-6 build -- whole GPU suite + smoke, then the c3 profile set (trace + PMC passes + judged line)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash $R/tools/gpu_check.sh r06x || exit 1
bash $R/tools/gpu_profile.sh r06x c3 || exit 1
echo r06x1 done
