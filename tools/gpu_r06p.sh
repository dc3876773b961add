#!/bin/bash
# r06p: the token-linear column-tile test over every tile
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06p
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest $R/tests/test_swin_unetr_gpu.py -m gpu -q -k "column_tiles or residual_epilogue or gelu_epilogue" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/t.log 2>&1
rc=$?; tail -2 $O/t.log; grep -E "^E |FAILED" $O/t.log | head -20; echo "rc $rc"
