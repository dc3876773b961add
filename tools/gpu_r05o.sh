# r05o: wgrad_brick2 two-set register prefetch (MMSEG_WGRAD_P2) -- bitwise test, c3 parity, c3 A/B; then the full suite
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r05o; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest $R/tests/test_kernels_gpu.py -x -q -k "p2_bitwise or conv3_fwd_dgrad_wgrad or wgrad_dma" --timeout 600 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/tests.log | head -20; exit 1; }
b() { n=$1; shift; timeout -k 10 600 env "$@" python3 $R/bench.py --steps 30 --warmup 5 --no-cpu-baseline --timer-steps 1 --timer-dump $O/timer_$n.json > $O/bench_$n.log 2>&1 || { tail -20 $O/bench_$n.log; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench_$n.log').read().strip().splitlines()[-1]); print('$n', d['ms_per_step'], d['value'])"; }
b p2 MMSEG_WGRAD_P2=1 && b nop2 MMSEG_WGRAD_P2=0 && b p2_b MMSEG_WGRAD_P2=1 && b nop2_b MMSEG_WGRAD_P2=0
python3 $R/tools/timer_families.py $O/timer_p2.json 6 && python3 $R/tools/timer_families.py $O/timer_nop2.json 6
bash $R/tools/gpu_check.sh r05o_check
