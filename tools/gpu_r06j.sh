#!/bin/bash
# r06j: GPU tests touching the token-linear GEMMs / window attention / small-volume norms after the tile changes
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06j
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest $R/tests/test_swin_unetr_gpu.py $R/tests/test_kernels_gpu.py $R/tests/test_model_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $O/t.log 2>&1
rc=$?
tail -3 $O/t.log
grep -E "^E |FAILED" $O/t.log | head -20
echo "rc $rc"
