#!/bin/bash
# A/B of one env knob on tools/convtbench.py shapes, rocprofv3-timed.  usage: bash tools/gpu_ctab.sh TAG KNOB "vals" shapes...
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=$1; KNOB=$2; VALS=$3; shift 3
O=$R/gpurun_out/$TAG
mkdir -p $O
for v in $VALS; do
  for sh in "$@"; do
    export $KNOB=$v
    timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t${v}_$sh -o t -- python3 $R/tools/convtbench.py --shape $sh > $O/t${v}_$sh.log 2>&1 || { tail -5 $O/t${v}_$sh.log; exit 1; }
    echo "== $KNOB=$v $sh"; python3 $R/tools/kstats.py $O/t${v}_$sh conv_gemm wgrad colsum reduce
  done
done
