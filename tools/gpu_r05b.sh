# r05b: KW=2 runtime-brick conv (12^3 / 6^3): kernel tests, convbench A/B KW=1 vs 2, c3 bench + DP rehearsal trace
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r05b; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest $R/tests/test_kernels_gpu.py $R/tests/test_swin_unetr_gpu.py -k "conv3_kernel_variants or b32 or window_attention" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/tests.log | head -20; exit 1; }
SH="4,12,128,256 4,12,256,256 4,6,256,512 4,6,512,512 2,12,512,256 2,12,256,256"
for kw in 1 2 1 2; do
  MMSEG_BRICKR_KW=$kw timeout -k 10 300 python3 $R/tools/convbench.py --shape $SH --only fwd,dgrad --iters 30 > $O/cb_kw$kw.log 2>&1 || { tail -5 $O/cb_kw$kw.log; exit 1; }
  echo "kw=$kw"; python3 -c "
import json,sys
for l in open('$O/cb_kw$kw.log'):
    if l.startswith('{'):
        d=json.loads(l); print(' ', d.get('shape'), d.get('op'), d.get('kernel'), d.get('us'))
"
done
timeout -k 10 600 python3 $R/bench.py --no-cpu-baseline --timer-dump $O/timer.json > $O/c3.log 2>&1 || { tail -20 $O/c3.log; exit 1; }
tail -1 $O/c3.log | cut -c1-200
MMSEG_BRICKR_KW=1 timeout -k 10 600 python3 $R/bench.py --no-cpu-baseline > $O/c3kw1.log 2>&1 || { tail -20 $O/c3kw1.log; exit 1; }
tail -1 $O/c3kw1.log | cut -c1-200
timeout -k 10 600 python3 $R/bench.py --no-cpu-baseline > $O/c3b.log 2>&1 || { tail -20 $O/c3b.log; exit 1; }
tail -1 $O/c3b.log | cut -c1-200
timeout -k 10 600 rocprofv3 -M --kernel-trace --output-format csv -d $O/dptrace -o prof -- python3 $R/bench.py --no-cpu-baseline --dp-rehearsal --steps 10 --warmup 3 --timer-steps 1 > $O/dptrace.log 2>&1 || { tail -20 $O/dptrace.log; exit 1; }
tail -1 $O/dptrace.log | cut -c1-200
timeout -k 10 600 python3 $R/bench.py --no-cpu-baseline --model swin_unetr --size 128 --batch 1 --steps 5 --warmup 2 > $O/c4.log 2>&1 || { tail -20 $O/c4.log; exit 1; }
tail -1 $O/c4.log | cut -c1-200
MMSEG_WINATTN_FWD1=0 timeout -k 10 600 python3 $R/bench.py --no-cpu-baseline --model swin_unetr --size 128 --batch 1 --steps 5 --warmup 2 > $O/c4old.log 2>&1 || { tail -20 $O/c4old.log; exit 1; }
tail -1 $O/c4old.log | cut -c1-200
echo done
