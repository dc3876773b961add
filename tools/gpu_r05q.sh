# r05q: paired-tap K tail (48 real of 64 channels) in brick2, templated zero-pad stores; tests + c4 A/B
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r05q; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest $R/tests/test_kernels_gpu.py $R/tests/test_swin_unetr_gpu.py -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/tests.log | head -20; exit 1; }
b() { n=$1; shift; timeout -k 10 600 env "$@" python3 $R/bench.py --model swin_unetr --size 128 --batch 1 --steps 10 --warmup 3 --no-cpu-baseline --timer-steps 1 --timer-dump $O/timer_$n.json > $O/bench_$n.log 2>&1 || { tail -20 $O/bench_$n.log; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench_$n.log').read().strip().splitlines()[-1]); print('$n', d['ms_per_step'], d['value'])"; }
b kt MMSEG_KTAIL16=1 && b nokt MMSEG_KTAIL16=0 && b nomu MMSEG_BRICK2_MINUNITS=0 && b kt_b MMSEG_KTAIL16=1
for n in kt nokt nomu; do python3 $R/tools/timer_families.py $O/timer_$n.json 8; done
