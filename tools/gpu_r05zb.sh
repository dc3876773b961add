# r05zb: 48-column tiles on the 8x8x8 LDS-DMA brick conv (MMSEG_BRICK8_BN48) with the 16x16x16 half-chunk tail (MMSEG_KTAIL16); conv + swin tests, c4 A/B
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r05zb; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest $R/tests/test_kernels_gpu.py $R/tests/test_swin_unetr_gpu.py -x -q -k "brick8 or conv3 or swin" --timeout 600 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/tests.log | head -20; exit 1; }
for v in on k0 b0 on; do
  e=""; [ $v = k0 ] && e="MMSEG_KTAIL16=0"; [ $v = b0 ] && e="MMSEG_BRICK8_BN48=0"
  env $e timeout -k 10 400 python3 $R/bench.py --model swin_unetr --size 128 --batch 1 --steps 10 --warmup 3 --no-cpu-baseline --timer-steps 1 --timer-dump $O/timer_$v.json > $O/bench_$v.log 2>&1 || { tail -20 $O/bench_$v.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/bench_$v.log').read().strip().splitlines()[-1]); print('$v c4', d['ms_per_step'])"
  python3 $R/tools/timer_families.py $O/timer_$v.json 60 | grep -E "conv3_brick|launches"
done
