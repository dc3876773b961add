#!/bin/bash
# 12^3 / 6^3 runtime-brick conv: 32-column tiles instead of a chunk split (MMSEG_BRICKR_BN32_BLK): microbench + c3 A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04v
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
S="4,12,128,256 4,12,256,256 4,6,256,512 4,6,512,512 2,12,512,256 2,12,256,256 2,24,256,128"
run() {
  echo "== $*"
  env "$@" timeout -k 10 120 python3 $R/tools/convbench.py --shape $S --only fwd,dgrad --iters 30 > $O/cb.log 2>&1 || { tail -20 $O/cb.log; exit 1; }
  python3 -c "
import json
for l in open('$O/cb.log'):
    if l.startswith('{'):
        d=json.loads(l); print(f\"{d['shape']:14s} {d['op']:6s} {d['kernel'][:40]:40s} {d['us']:8.1f} us {d['tflops']:7.1f} TF/s\")"
}
run MMSEG_BRICKR_BN32_BLK=0
run MMSEG_BRICKR_BN32_BLK=256
AB_STEPS=40 bash $R/tools/gpu_ab.sh r04v_ab - MMSEG_BRICKR_BN32_BLK=256 MMSEG_BRICKR_BN32_BLK=200 - MMSEG_BRICKR_BN32_BLK=256 MMSEG_BRICKR_BN32_BLK=200
