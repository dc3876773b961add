# r05r: few-unit brick2 shapes on the runtime brick (MMSEG_BRICK2_MINUNITS A/B), templated zero-pad stores; c4 + c3
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r05r; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest $R/tests/test_kernels_gpu.py $R/tests/test_swin_unetr_gpu.py -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/tests.log | head -20; exit 1; }
b() { n=$1; shift; timeout -k 10 600 env "$@" python3 $R/bench.py $BA --no-cpu-baseline --timer-steps 1 --timer-dump $O/timer_$n.json > $O/bench_$n.log 2>&1 || { tail -20 $O/bench_$n.log; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench_$n.log').read().strip().splitlines()[-1]); print('$n', d['ms_per_step'], d['value'])"; }
BA="--model swin_unetr --size 128 --batch 1 --steps 10 --warmup 3"
b mu MMSEG_BRICK2_MINUNITS=128 && b nomu MMSEG_BRICK2_MINUNITS=0 && b mu_b MMSEG_BRICK2_MINUNITS=128
BA="--steps 30 --warmup 5"
b c3 MMSEG_BRICK2_MINUNITS=128 && b c3_nomu MMSEG_BRICK2_MINUNITS=0
for n in mu nomu; do python3 $R/tools/timer_families.py $O/timer_$n.json 10; done
