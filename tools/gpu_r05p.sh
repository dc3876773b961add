# r05p: in_bwd_apply zero-pad store as its own instantiation (c3 regression check), c3 + c4 bench, IN tests
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r05p; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest $R/tests/test_swin_unetr_gpu.py $R/tests/test_kernels_gpu.py -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/tests.log | head -20; exit 1; }
b() { n=$1; shift; timeout -k 10 600 python3 $R/bench.py "$@" --no-cpu-baseline --timer-steps 1 --timer-dump $O/timer_$n.json > $O/bench_$n.log 2>&1 || { tail -20 $O/bench_$n.log; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench_$n.log').read().strip().splitlines()[-1]); print('$n', d['ms_per_step'], d['value'])"; }
b c3 --steps 30 --warmup 5 && b c3_b --steps 30 --warmup 5 && b c4 --model swin_unetr --size 128 --batch 1 --steps 10 --warmup 3
python3 $R/tools/timer_families.py $O/timer_c3.json 8
