# r05z5: 48-row weight-gradient tiles for SwinUNETR's padded 64-row levels (phase bit 8) and the 128x96 point-GEMM
# tile; wgrad + swin tests, c4 A/B of each
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r05z5; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest $R/tests/test_kernels_gpu.py $R/tests/test_swin_unetr_gpu.py -x -q -k "wgrad or swin" --timeout 600 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/tests.log | head -20; exit 1; }
for v in on pad0 bn0 pd0 sw0 on; do
  e=""; [ $v = pad0 ] && e="MMSEG_WGRAD_PAD16=0"; [ $v = bn0 ] && e="MMSEG_POINT_BN96=0"; [ $v = pd0 ] && e="MMSEG_WGRAD_PDIRECT=0"; [ $v = sw0 ] && e="MMSEG_WINATTN_SWZ=0"
  env $e timeout -k 10 400 python3 $R/bench.py --model swin_unetr --size 128 --batch 1 --steps 10 --warmup 3 --no-cpu-baseline --timer-steps 1 --timer-dump $O/timer_c4_$v.json > $O/bench_c4_$v.log 2>&1 || { tail -20 $O/bench_c4_$v.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/bench_c4_$v.log').read().strip().splitlines()[-1]); print('$v c4', d['ms_per_step'], d['value'])"
  python3 $R/tools/timer_families.py $O/timer_c4_$v.json 60 | grep -E "wgrad_dma|point|reduce_batch|winattn|launches"
done
