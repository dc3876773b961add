#!/bin/bash
# brick6 timing-probe variants (libmmseg_hip_probe.so): full / MFMA + fragment reads / MFMA only
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-b6dbg}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for d in 0 1 2 3 0; do
  MMSEG_BRICK6_DBG=$d timeout -k 10 120 python3 -u $R/tools/convbench.py --probe --iters 30 --only fwd,fwdn --shape 2,96,32,32 > $O/cb.log 2>&1 || { tail -20 $O/cb.log; exit 1; }
  echo "== DBG $d"; grep -v amdgpu.ids $O/cb.log | grep -v "^  probe"
done
