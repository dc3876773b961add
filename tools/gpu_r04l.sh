#!/bin/bash
# r04l: kernel / model / swin GPU tests (forced 24^3 grouping, transposed-conv index math), bench with a timer
# dump, then A/B of the forced grouping and the runtime-brick slots
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04l
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest $R/tests/test_model_gpu.py::test_grouped_modalities_match_per_modality $R/tests/test_kernels_gpu.py $R/tests/test_model_gpu.py $R/tests/test_swin_unetr_gpu.py -m gpu -q -s --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
grep -E "grouped from level|largest gradient" $O/tests.log | cut -c1-400
[ $rc -ne 0 ] && [ $rc -ne 1 ] && { echo "tests ended with $rc"; tail -20 $O/tests.log; exit 1; }
[ $rc -eq 1 ] && grep -E "^FAILED|^E " $O/tests.log | head -20
timeout -k 10 600 python3 $R/bench.py --timer-dump $O/timer.json --no-cpu-baseline > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-200
python3 $R/tools/timer_dump.py $O/timer.json 10 | head -45
AB_STEPS=40 bash $R/tools/gpu_ab.sh r04l_ab - MMSEG_GROUP_FORCE_R=1 MMSEG_BRICKR_SLOTS=128 - MMSEG_GROUP_FORCE_R=1 MMSEG_BRICKR_SLOTS=128 - MMSEG_GROUP_FORCE_R=1
