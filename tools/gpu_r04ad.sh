#!/bin/bash
# grouped 48^3 / 24^3 InstanceNorm statistics from the runtime-brick epilogue (MMSEG_GROUP_STATS): tests + c3/c5 A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04ad
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest "$R/tests/test_model_gpu.py" "$R/tests/test_step_graph_gpu.py" "$R/tests/test_fullsize_gpu.py::test_fullsize_step_pinned_to_fp64_oracle" -k "group or pinned or bench or dual" -m gpu -v -s --timeout 600 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
grep -E "pinned fp64" $O/tests.log | cut -c1-250
[ $rc -ne 0 ] && { grep -E "^E |FAILED" $O/tests.log | head -20; exit 1; }
AB_STEPS=40 bash $R/tools/gpu_ab.sh r04ad_ab - MMSEG_GROUP_STATS=0 - MMSEG_GROUP_STATS=0 || exit 1
AB_STEPS=30 bash $R/tools/gpu_ab.sh r04ad_c5 "--modalities=CT,PET,MRI --loss=tversky" "MMSEG_GROUP_STATS=0 --modalities=CT,PET,MRI --loss=tversky"
