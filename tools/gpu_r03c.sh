#!/bin/bash
# brick8 check + A/B: kernel-variant tests, then convbench of the 48^3 layers with MMSEG_BRICK8 0 / 1, then the
# bench with each.  usage: bash tools/gpu_r03c.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r03c}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest $R/tests/test_kernels_gpu.py -m gpu -k "variants or b32" -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" $O/tests.log | head -20; exit 1; fi
for v in 0 1; do
  MMSEG_BRICK8=$v timeout -k 10 300 python3 $R/tools/convbench.py --shape 2,48,32,64 2,48,64,64 2,48,128,64 2,96,64,32 2,96,32,64 2,48,64,32 2,24,128,128 --only fwd,dgrad > $O/cb_$v.log 2>&1 || { tail -5 $O/cb_$v.log; exit 1; }
  echo "== MMSEG_BRICK8=$v"; grep '^{' $O/cb_$v.log | cut -c1-200
done
for v in 0 1; do
  MMSEG_BRICK8=$v timeout -k 10 600 python3 $R/bench.py --no-cpu-baseline > $O/bench_$v.log 2>&1 || { tail -20 $O/bench_$v.log; exit 1; }
  echo "== bench MMSEG_BRICK8=$v"; tail -1 $O/bench_$v.log | cut -c1-300
done
