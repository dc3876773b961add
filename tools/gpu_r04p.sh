#!/bin/bash
# runtime-brick conv microbench at the grouped 48^3 / 24^3 shapes (N = 2 modalities x 2 samples): variants
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04p
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
S="4,48,32,64 4,48,64,64 4,24,64,128 4,24,128,128"
run() {
  echo "== $*"
  env "$@" timeout -k 10 120 python3 $R/tools/convbench.py --shape $S --only fwd,dgrad --iters 30 > $O/cb.log 2>&1 || { tail -20 $O/cb.log; exit 1; }
  python3 -c "
import json
for l in open('$O/cb.log'):
    if l.startswith('{'):
        d=json.loads(l); print(f\"{d['shape']:14s} {d['op']:6s} {d['kernel'][:40]:40s} {d['us']:8.1f} us {d['tflops']:7.1f} TF/s\")"
}
run MMSEG_BRICK=3
run MMSEG_BRICK=3 MMSEG_BRICKR_CT488=0
run MMSEG_BRICK=3 MMSEG_BRICKR_SLOTS=512
run MMSEG_BRICK=3 MMSEG_BRICKR_SLOTS=128
run MMSEG_BRICK=2
