# r05f: c4 -- trimmed one-pass attention forward, wide-tile token linears: tests + bench A/B
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r05f; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest $R/tests/test_swin_unetr_gpu.py $R/tests/test_swin_attention_gpu.py -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/tests.log | head -20; exit 1; }
for v in 1 0 1 0; do
MMSEG_POINT_WIDE=$v timeout -k 10 600 python3 $R/bench.py --no-cpu-baseline --model swin_unetr --size 128 --batch 1 --steps 5 --warmup 2 > $O/c4_$v.log 2>&1 || { tail -20 $O/c4_$v.log; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/c4_$v.log').read().strip().splitlines()[-1])
print('WIDE=$v', d['ms_per_step'], {k: v['ms_per_step'] for k, v in d['kernel_families'].items() if 'point' in k or 'winattn' in k})
"
done
echo done
