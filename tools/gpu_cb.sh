#!/bin/bash
# GPU tests (one process) then conv microbench variants: bash tools/gpu_cb.sh TAG "ENV=.. ENV2=.." ["ENV=.."...]
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=${1:-cb}; shift
O=$R/gpurun_out/$TAG
mkdir -p $O
if [ -z "$NOTEST" ]; then
timeout -k 10 600 python3 -m pytest $R/tests -m gpu -q -x > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log
[ $rc -le 1 ] || exit 1
fi
i=0
for v in "$@"; do
  i=$((i+1))
  env $v timeout -k 10 300 python3 $R/tools/convbench.py $CB_ARGS > $O/conv_$i.log 2>&1 || { tail -5 $O/conv_$i.log; exit 1; }
  echo "== $v"; grep '^{' $O/conv_$i.log
done
