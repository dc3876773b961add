#!/bin/bash
# r06a: whole GPU suite on the round-6 fixes (tile-pitch checks, stem Co=48 routing, DP capture reset, whole-row
# padding, c4 sliding window at size), the c1 drift diagnosis (2dc10ed's routing off), c4 inference + bench lines
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06a
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest $R/tests -m gpu -q -s --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
rc=$?
tail -2 $O/gpu_tests.log
grep -E "^E |FAILED|held-out|free-running|sliding window|unet48" $O/gpu_tests.log | head -30
[ $rc -gt 1 ] && { echo "suite rc $rc"; exit 1; }
MMSEG_BRICK2_MINUNITS=0 timeout -k 10 600 python3 -u -m pytest $R/tests/test_dice_heldout_gpu.py -q -s --timeout 300 --timeout-method thread -p no:cacheprovider -k "matches_reference or free_running" > $O/dice_minunits0.log 2>&1
rc=$?
grep -E "held-out|free-running|passed|failed" $O/dice_minunits0.log
[ $rc -gt 1 ] && exit 1
cd $R
timeout -k 10 600 python3 bench.py --model swin_unetr --size 128 --batch 1 --infer --steps 3 --warmup 1 > $O/infer_c4.log 2>&1 || { tail -20 $O/infer_c4.log; exit 1; }
tail -1 $O/infer_c4.log
timeout -k 10 600 python3 bench.py --model swin_unetr --size 128 --batch 1 --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_c4.log 2>&1 || { tail -20 $O/bench_c4.log; exit 1; }
tail -1 $O/bench_c4.log | cut -c1-1500
timeout -k 10 600 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_c3.log 2>&1 || { tail -20 $O/bench_c3.log; exit 1; }
tail -1 $O/bench_c3.log | cut -c1-1200
echo r06a done
