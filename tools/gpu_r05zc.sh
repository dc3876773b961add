# r05zc: precomputed staging offsets in the 32-co brick weight gradient (MMSEG_WGRAD_B2_REL); wgrad tests, c3 A/B
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r05zc; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest $R/tests/test_kernels_gpu.py -x -q -k "wgrad" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/tests.log | head -20; exit 1; }
for p in 1 0 1 0; do
  MMSEG_WGRAD_B2_REL=$p timeout -k 10 300 python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --timer-steps 1 --timer-dump $O/timer_$p.json > $O/bench_$p.log 2>&1 || { tail -20 $O/bench_$p.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/bench_$p.log').read().strip().splitlines()[-1]); print('rel $p c3', d['ms_per_step'], d['roofline']['kernel'], d['roofline']['avg_launch_ms'], d['roofline']['frac'])"
done
