#!/bin/bash
# r06z2: head backward (per-group data gradient, padded-group weight-gradient partials) -- head tests, then the
# c4 profile set (families, PMC) and bench line
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06z2
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest $R/tests/test_swin_unetr_gpu.py $R/tests/test_kernels_gpu.py -m gpu -x -q \
  -k "head or train_step" --timeout 240 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
[ $rc -ne 0 ] && { grep -E "^E " $O/tests.log | head -20; exit 1; }
bash $R/tools/gpu_profile.sh r06z2 c4 --model swin_unetr --size 128 --batch 1 || exit 1
echo r06z2 done
