#!/bin/bash
# grouped levels read the fused gradient modulo N (no M-fold copy, MMSEG_GROUP_REPLICATE=0); brick6 INP writes
# its own zero partials (no memset): tests + c3 A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04aa
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest "$R/tests/test_model_gpu.py" "$R/tests/test_step_graph_gpu.py" "$R/tests/test_fullsize_gpu.py::test_fullsize_step_pinned_to_fp64_oracle" -k "head_in_partials or group or pinned or bench or dual" -m gpu -v -s --timeout 600 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
grep -E "pinned fp64" $O/tests.log | cut -c1-250
[ $rc -ne 0 ] && { grep -E "^E |FAILED" $O/tests.log | head -20; exit 1; }
AB_STEPS=40 bash $R/tools/gpu_ab.sh r04aa_ab - MMSEG_GROUP_REPLICATE=1 - MMSEG_GROUP_REPLICATE=1
