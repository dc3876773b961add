#!/bin/bash
# r06zc: row-group passes (res_apply / lrelu_bwd) on at most 2,048 blocks (in-tree) or 4,096 instead of up to 16,384
# (one 4-row round per thread, each paying its 32-float statistics preload): the c4 step per build against the
# previous one, interleaved, per-family timer; then the whole GPU suite + smoke on the in-tree build.  Result:
# res_apply 0.769 / 0.766 / 0.751 ms per step (16,384 / 2,048 / 4,096 blocks): not kept, reverted (profiles/r06zc_*)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06zc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P=$R/multimodal-organ-segmentation_amd
i=0
for v in prev r2048 r4096 prev r2048 r4096; do
  lib=$P/libmmseg_hip_$v.so; [ $v = r2048 ] && lib=$P/libmmseg_hip.so
  timeout -k 10 400 python3 $R/tools/benchlib.py $lib --model swin_unetr --size 128 --batch 1 --steps 20 --warmup 5 --no-cpu-baseline --timer-steps 2 > $O/c4_${v}_$i.log 2>&1 || { tail -20 $O/c4_${v}_$i.log; exit 1; }
  tail -1 $O/c4_${v}_$i.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); f=d['kernel_families']
print('== c4 $v', d['ms_per_step'], d['loss'], {k: f[k]['ms_per_step'] for k in f if k.startswith('res_apply') or k.startswith('lrelu_bwd_k')})"
  i=$((i+1))
done
bash $R/tools/gpu_check.sh r06zc || exit 1
echo r06zc done
