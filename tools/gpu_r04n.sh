#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04n
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest "$R/tests/test_fullsize_gpu.py::test_fullsize_step_pinned_to_fp64_oracle" -k force -m gpu -v -s --timeout 600 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
grep -E "pinned fp64" $O/tests.log | cut -c1-400
[ $rc -ne 0 ] && { grep -E "^E |FAILED" $O/tests.log | head -20; exit 1; }
AB_STEPS=40 bash $R/tools/gpu_ab.sh r04n_ab - MMSEG_GROUP_FORCE_R=1 - MMSEG_GROUP_FORCE_R=1
