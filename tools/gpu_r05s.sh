# r05s: 48-column stem for SwinUNETR encoder1 conv1; swin + kernel + model tests; c4 bench
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r05s; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest $R/tests/test_swin_unetr_gpu.py $R/tests/test_kernels_gpu.py -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/tests.log | head -20; exit 1; }
grep -E "c4 128|pinned" $O/tests.log | head
b() { n=$1; shift; timeout -k 10 600 env "$@" python3 $R/bench.py $BA --no-cpu-baseline --timer-steps 1 --timer-dump $O/timer_$n.json > $O/bench_$n.log 2>&1 || { tail -20 $O/bench_$n.log; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench_$n.log').read().strip().splitlines()[-1]); print('$n', d['ms_per_step'], d['value'])"; }
BA="--model swin_unetr --size 128 --batch 1 --steps 10 --warmup 3"
b c4 MMSEG_STEM=1 && b c4_nostem MMSEG_STEM=0 && b c4_b MMSEG_STEM=1
for n in c4 c4_nostem; do python3 $R/tools/timer_families.py $O/timer_$n.json 40 | grep -E "stem|conv3,128|wgrad_kernel<conv3|launches"; done
