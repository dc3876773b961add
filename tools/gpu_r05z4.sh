# r05z4: 16-B stores in the channel-major split reduce (MMSEG_WRED_V4); wgrad kernel tests, c4 / c3 A/B
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r05z4; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest $R/tests/test_kernels_gpu.py -x -q -k "wgrad" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/tests.log | head -20; exit 1; }
for v in 1 0; do
  MMSEG_WRED_V4=$v timeout -k 10 400 python3 $R/bench.py --model swin_unetr --size 128 --batch 1 --steps 10 --warmup 3 --no-cpu-baseline --timer-steps 1 --timer-dump $O/timer_c4_$v.json > $O/bench_c4_$v.log 2>&1 || { tail -20 $O/bench_c4_$v.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/bench_c4_$v.log').read().strip().splitlines()[-1]); print('v4 $v c4', d['ms_per_step'], d['value'])"
  python3 $R/tools/timer_families.py $O/timer_c4_$v.json 60 | grep -E "wgrad_reduce|launches"
  MMSEG_WRED_V4=$v timeout -k 10 300 python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --timer-steps 1 --timer-dump $O/timer_c3_$v.json > $O/bench_c3_$v.log 2>&1 || { tail -20 $O/bench_c3_$v.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/bench_c3_$v.log').read().strip().splitlines()[-1]); print('v4 $v c3', d['ms_per_step'], d['value'])"
  python3 $R/tools/timer_families.py $O/timer_c3_$v.json 60 | grep -E "wgrad_reduce|launches"
done
