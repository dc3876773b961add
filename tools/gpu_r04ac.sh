#!/bin/bash
# runtime-brick 4x8x8 (grouped 48^3 / 24^3) with tap-ahead fragment reads (MMSEG_BRICKR_PF488)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04ac
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
run MMSEG_BRICK=3 MMSEG_BRICKR_PF488=0
run MMSEG_BRICK=3 MMSEG_BRICKR_PF488=1
timeout -k 10 300 python3 -u -m pytest "$R/tests/test_kernels_gpu.py" -k "b32_halo or kernel_variants" -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests_pf0.log 2>&1; tail -1 $O/tests_pf0.log
MMSEG_BRICKR_PF488=1 timeout -k 10 300 python3 -u -m pytest "$R/tests/test_kernels_gpu.py" -k "b32_halo or kernel_variants" -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests_pf1.log 2>&1; tail -1 $O/tests_pf1.log
AB_STEPS=40 bash $R/tools/gpu_ab.sh r04ac_ab - MMSEG_BRICKR_PF488=1 - MMSEG_BRICKR_PF488=1
