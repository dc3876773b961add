#!/bin/bash
# r04j: forced 24^3 grouping tests + a three-round A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04j
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest $R/tests/test_model_gpu.py::test_grouped_modalities_match_per_modality -m gpu -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
grep -E "grouped from level" $O/tests.log
[ $rc -ne 0 ] && { grep -E "^E |Error" $O/tests.log | head -20; exit 1; }
AB_STEPS=40 bash $R/tools/gpu_ab.sh r04j_ab - MMSEG_GROUP_FORCE_R=1 - MMSEG_GROUP_FORCE_R=1 - MMSEG_GROUP_FORCE_R=1
