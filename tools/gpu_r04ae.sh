#!/bin/bash
# grouped-test coverage of MMSEG_GROUP_STATS=1 (off by default) + the grouped / pinned tests on the final tree
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04ae
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest "$R/tests/test_model_gpu.py" -k "group" -m gpu -v -s --timeout 600 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
grep -E "grouped from level" $O/tests.log | cut -c1-200
[ $rc -ne 0 ] && { grep -E "^E |FAILED" $O/tests.log | head -20; exit 1; }
echo ok
