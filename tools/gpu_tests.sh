#!/bin/bash
# run selected GPU test files.  usage: bash tools/gpu_tests.sh TAG test_file...
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=${1:-t}; shift
O=$R/gpurun_out/$TAG
mkdir -p $O
ARGS=""
for f in "$@"; do ARGS="$ARGS $R/tests/$f"; done
timeout -k 10 600 python3 -u -m pytest $ARGS -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|error" $O/tests.log | tail -40
tail -3 $O/tests.log
exit $rc
