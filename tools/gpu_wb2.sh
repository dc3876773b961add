#!/bin/bash
# wgrad_brick2 with the next brick's staging between the dy planes (MMSEG_WGRAD_IL) vs after them
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-wb2}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest $R/tests/test_kernels_gpu.py $R/tests/test_model_gpu.py -q -x --timeout 300 --timeout-method thread -p no:cacheprovider -k "variants or deferred_conv_norm or conv3_fwd_dgrad_wgrad" > $O/tests.log 2>&1
rc=$?
tail -2 $O/tests.log
[ $rc -ne 0 ] && { grep -E "^E |Error" $O/tests.log | head -8; exit $rc; }
for v in "MMSEG_WGRAD_IL=0" "MMSEG_WGRAD_IL=1" "MMSEG_WGRAD_IL=0" "MMSEG_WGRAD_IL=1"; do
  env $v MMSEG_WGRAD_DMA=0 timeout -k 10 120 python3 -u $R/tools/convbench.py --iters 30 --only wgrad,wgradn --shape 2,96,32,32 > $O/cb.log 2>&1 || { tail -20 $O/cb.log; exit 1; }
  echo "== $v $(grep -v amdgpu.ids $O/cb.log | tr '\n' ' ')"
done
timeout -k 10 300 python3 -u $R/tools/kbench.py --variants "MMSEG_WGRAD_IL=0,1" --rounds 5 --steps 10 > $O/kb.log 2>&1 || { tail -20 $O/kb.log; exit 1; }
grep variant $O/kb.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); f=d['families']
    print(d['variant'], d['median_ms'], d['min_ms'], {k:v for k,v in f.items() if 'wgrad_brick2' in k})"
