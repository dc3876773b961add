#!/bin/bash
# Block-timeline probes of the brick conv kernels (libmmseg_hip_probe.so; tools/convbench.py --probe).
# usage: bash tools/gpu_probe.sh TAG [SHAPES...]; env knobs pass through
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-probe}
mkdir -p $O
shift
SH=${@:-2,48,64,64 2,48,32,64}
MMSEG_BRICK8=0 timeout -k 10 180 python3 -u $R/tools/convbench.py --probe --iters 10 --only fwd,dgrad --shape $SH > $O/b2.log 2>&1 || { tail -20 $O/b2.log; exit 1; }
cat $O/b2.log | grep -v amdgpu.ids
MMSEG_BRICK8=2 MMSEG_BRICK8_MINBLK=0 timeout -k 10 180 python3 -u $R/tools/convbench.py --probe --iters 10 --only fwd,dgrad --shape $SH > $O/b8.log 2>&1 || { tail -20 $O/b8.log; exit 1; }
cat $O/b8.log | grep -v amdgpu.ids
