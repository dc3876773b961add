#!/bin/bash
# convbench A/B over environment variants: bash tools/gpu_cbab.sh TAG "SHAPES" "VAR=1 ..." "-" ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; SH=$2; shift 2
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for v in "$@"; do
  e=$v; [ "$e" = "-" ] && e=""
  env $e timeout -k 10 300 python3 $R/tools/convbench.py --iters ${CB_ITERS:-20} --only ${CB_OPS:-fwd,dgrad} --shape $SH > $O/cb_$i.log 2>&1 || { tail -20 $O/cb_$i.log; exit 1; }
  echo "== [$v]"; python3 $R/tools/cbfmt.py < $O/cb_$i.log
  i=$((i+1))
done
