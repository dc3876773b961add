#!/bin/bash
# r04k: kernel + model tests, then the bench with a timer dump
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04k
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest $R/tests/test_kernels_gpu.py $R/tests/test_model_gpu.py $R/tests/test_swin_unetr_gpu.py -m gpu -q -s --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
[ $rc -ne 0 ] && { grep -E "^E |Error|FAILED" $O/tests.log | head -20; exit 1; }
timeout -k 10 600 python3 $R/bench.py --timer-dump $O/timer.json --no-cpu-baseline > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-200
python3 $R/tools/timer_dump.py $O/timer.json 10 | head -45
AB_STEPS=40 bash $R/tools/gpu_ab.sh r04k_ab - MMSEG_BRICKR_SLOTS=128 MMSEG_BRICKR_SLOTS=64 - MMSEG_BRICKR_SLOTS=128 MMSEG_BRICKR_SLOTS=64
