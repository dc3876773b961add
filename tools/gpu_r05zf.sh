# r05zf: 128x128 point-GEMM tile for 128 / 256-column 1x1 GEMMs over many rows (MMSEG_POINT_BN128); swin tests, c4 A/B
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r05zf; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest $R/tests/test_swin_unetr_gpu.py -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/tests.log | head -20; exit 1; }
for v in 1 0 1 0; do
  MMSEG_POINT_BN128=$v timeout -k 10 400 python3 $R/bench.py --model swin_unetr --size 128 --batch 1 --steps 10 --warmup 3 --no-cpu-baseline --timer-steps 1 --timer-dump $O/timer_$v.json > $O/bench_$v.log 2>&1 || { tail -20 $O/bench_$v.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/bench_$v.log').read().strip().splitlines()[-1]); print('bn128 $v c4', d['ms_per_step'])"
  python3 $R/tools/timer_families.py $O/timer_$v.json 60 | grep -E "point|launches"
done
