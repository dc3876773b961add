#!/bin/bash
# brick5 (96^3 32->32) phase stamps (libmmseg_hip_probe.so, MMSEG_BRICK5_DBG) and the step's variants timed.
# usage: bash tools/gpu_b5probe.sh TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-b5probe}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 python3 -u $R/tools/convbench.py --iters 20 --only fwd,fwdn,dgrad,dgradin --shape 2,96,32,32 > $O/times.log 2>&1 || { tail -20 $O/times.log; exit 1; }
grep -v amdgpu.ids $O/times.log
for dma in 0 1; do
  MMSEG_BRICK5_DMA=$dma MMSEG_BRICK5_DBG=1 timeout -k 10 120 python3 -u $R/tools/convbench.py --probe --iters 3 --only fwd,fwdn --shape 2,96,32,32 > $O/probe_dma$dma.log 2>&1 || { tail -20 $O/probe_dma$dma.log; exit 1; }
  echo "== DMA $dma"; grep -v amdgpu.ids $O/probe_dma$dma.log | grep -v "^  probe" | head -24
done
