#!/bin/bash
# end-of-round check of the committed tree: the whole GPU suite, then smoke()
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-check}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest $R/tests -m gpu -q -s --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
rc=$?
tail -2 $O/gpu_tests.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED" $O/gpu_tests.log | head -20; exit 1; }
cd $R && timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
rc=$?
tail -3 $O/smoke.log
exit $rc
