#!/bin/bash
# A/B one env knob on convbench shapes in one GPU call.  usage: bash tools/gpu_cbab.sh TAG KNOB "vals" shapes...
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=$1; KNOB=$2; VALS=$3; shift 3
O=$R/gpurun_out/$TAG
mkdir -p $O
for v in $VALS; do
  env $KNOB=$v timeout -k 10 300 python3 $R/tools/convbench.py --shape "$@" > $O/$KNOB.$v.jsonl 2>&1 || { echo "fail $v"; tail -5 $O/$KNOB.$v.jsonl; exit 1; }
  echo "== $KNOB=$v"; grep shape $O/$KNOB.$v.jsonl
done
