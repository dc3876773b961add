#!/bin/bash
# r06z9: head backward (SwinUNETR's 48 / 64-channel rows) with one dlogits load per lane and voxel, the voxel's
# other classes taken by cross-lane reads: head tests, the c4 step against the previous build
# (libmmseg_hip_prev.so, interleaved, per-family timer), then the whole GPU suite + smoke on the new build.
# Result: weight-gradient partial 112 -> 158 us, data gradient 135 -> 132 us, c4 slower: not kept, reverted
# (profiles/r06z9_*)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06z9
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest $R/tests/test_swin_unetr_gpu.py $R/tests/test_kernels_gpu.py -m gpu -x -q \
  -k "head or train_step" --timeout 240 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
[ $rc -ne 0 ] && { grep -E "^E " $O/tests.log | head -20; exit 1; }
P=$R/multimodal-organ-segmentation_amd
i=0
for v in prev new prev new; do
  lib=$P/libmmseg_hip.so; [ $v = prev ] && lib=$P/libmmseg_hip_prev.so
  timeout -k 10 400 python3 $R/tools/benchlib.py $lib --model swin_unetr --size 128 --batch 1 --steps 20 --warmup 5 --no-cpu-baseline --timer-steps 2 > $O/c4_${v}_$i.log 2>&1 || { tail -20 $O/c4_${v}_$i.log; exit 1; }
  tail -1 $O/c4_${v}_$i.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); f=d['kernel_families']
print('== c4 $v', d['ms_per_step'], {k: f[k]['ms_per_step'] for k in f if 'head' in k})"
  i=$((i+1))
done
bash $R/tools/gpu_check.sh r06z9 || exit 1
echo r06z9 done
