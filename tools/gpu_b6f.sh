#!/bin/bash
# brick6 INP (data gradient with the InstanceNorm-backward partials) vs brick5's: parity, convbench, step A/B
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-b6f}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest $R/tests/test_kernels_gpu.py $R/tests/test_model_gpu.py $R/tests/test_fullsize_gpu.py -q -x --timeout 300 --timeout-method thread -p no:cacheprovider -k "variants or deferred_conv_norm or step_bitwise or head_in_partials or fullsize_training" > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
[ $rc -ne 0 ] && { grep -E "^E " $O/tests.log | head -5; exit $rc; }
for v in "MMSEG_BRICK6_INP=0" "MMSEG_BRICK6_INP=1" "MMSEG_BRICK6_INP=0" "MMSEG_BRICK6_INP=1"; do
  env $v timeout -k 10 120 python3 -u $R/tools/convbench.py --iters 30 --only dgradin --shape 2,96,32,32 > $O/cb.log 2>&1 || { tail -20 $O/cb.log; exit 1; }
  echo "== $v $(grep -v amdgpu.ids $O/cb.log)"
done
timeout -k 10 300 python3 -u $R/tools/kbench.py --variants "MMSEG_BRICK6_INP=0,1" --rounds 5 --steps 10 > $O/kb.log 2>&1 || { tail -20 $O/kb.log; exit 1; }
grep variant $O/kb.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); f=d['families']
    print(d['variant'], d['median_ms'], d['min_ms'], {k:v for k,v in f.items() if 'brick5' in k or 'brick6' in k})"
