#!/bin/bash
# brick6 block timeline (convbench --probe) and phase stamps (MMSEG_BRICK5_DBG routes to brick6's DBG=4 variant)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-b6st}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 python3 -u $R/tools/convbench.py --probe --iters 20 --only fwd,fwdn --shape 2,96,32,32 > $O/tl.log 2>&1 || { tail -20 $O/tl.log; exit 1; }
grep -v amdgpu.ids $O/tl.log
MMSEG_BRICK5_DBG=1 timeout -k 10 120 python3 -u $R/tools/convbench.py --probe --iters 2 --only fwd --shape 2,96,32,32 > $O/st_fwd.log 2>&1 || { tail -20 $O/st_fwd.log; exit 1; }
grep "dbg slot" $O/st_fwd.log | tail -4
