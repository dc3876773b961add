#!/bin/bash
# End-of-round GPU call: full GPU suite, bench + rocprofv3 trace + PMC passes (tools/gpu_round.sh), then the bench
# line of every BASELINE config (tools/gpu_configs.sh).  usage: bash tools/gpu_final.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-final}
bash $R/tools/gpu_round.sh $T || exit 1
bash $R/tools/gpu_configs.sh ${T}_cfg || exit 1
echo final done
