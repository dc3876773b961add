#!/bin/bash
# convbench over values of one knob (no tests, no bench): bash tools/gpu_cbvar.sh TAG KNOB "v1 v2 .." [shapes] [ops]
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=$1; KNOB=$2; VALS=$3; SHAPES=${4:-"2,96,32,32"}; OPS=${5:-fwd}
O=$R/gpurun_out/$TAG
mkdir -p $O
for v in $VALS; do
  env $KNOB=$v timeout -k 10 300 python3 $R/tools/convbench.py --shape $SHAPES --only $OPS > $O/conv_$v.log 2>&1 || { tail $O/conv_$v.log; exit 1; }
  echo "== $KNOB=$v"; grep shape $O/conv_$v.log
done
