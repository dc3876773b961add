#!/bin/bash
# wgrad_dma: previous build (libmmseg_hip_old.so) vs this one with / without the interleaved DMA issue (IL)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-wd}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
SH="2,48,64,64 2,24,128,128 2,48,128,64 2,96,64,32"
for rep in 1 2; do
  for v in "old" "IL=0" "IL=1"; do
    if [ $v = old ]; then a="--lib libmmseg_hip_old.so"; e=""; else a=""; e="MMSEG_WGRAD_DMA_$v"; fi
    env $e timeout -k 10 120 python3 -u $R/tools/convbench.py $a --iters 30 --only wgrad --shape $SH > $O/cb.log 2>&1 || { tail -20 $O/cb.log; exit 1; }
    echo "== $v"; grep -v amdgpu.ids $O/cb.log | python3 -c "
import json,sys
print('  '.join(f\"{d['shape']}:{d['us']}\" for d in map(json.loads, sys.stdin)))"
  done
done
timeout -k 10 600 python3 -u -m pytest $R/tests/test_kernels_gpu.py $R/tests/test_model_gpu.py -q -x --timeout 300 --timeout-method thread -p no:cacheprovider -k "variants or deferred_conv_norm or step_bitwise or conv3_fwd_dgrad_wgrad" > $O/tests.log 2>&1
rc=$?
tail -2 $O/tests.log
[ $rc -ne 0 ] && { grep -E "^E " $O/tests.log | head -5; exit $rc; }
timeout -k 10 300 python3 -u $R/tools/kbench.py --variants "MMSEG_WGRAD_DMA_IL=0,1" --rounds 5 --steps 10 > $O/kb.log 2>&1 || { tail -20 $O/kb.log; exit 1; }
grep variant $O/kb.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); f=d['families']
    print(d['variant'], d['median_ms'], d['min_ms'], {k:v for k,v in f.items() if 'wgrad_dma' in k})"
