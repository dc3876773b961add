#!/bin/bash
# r06zb: head data-gradient grid cap (8,192 blocks before; 1,024 / 2,048 (in-tree build) / 4,096 blocks, i.e. 8 to
# 64 voxels per lane): head tests on the in-tree build, then the c4 step per build, interleaved, per-family timer;
# then the whole GPU suite + smoke on the in-tree build
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06zb
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest $R/tests/test_swin_unetr_gpu.py $R/tests/test_kernels_gpu.py -m gpu -x -q \
  -k "head or train_step" --timeout 240 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
[ $rc -ne 0 ] && { grep -E "^E " $O/tests.log | head -20; exit 1; }
P=$R/multimodal-organ-segmentation_amd
i=0
for v in prev g1024 g2048 g4096 prev g1024 g2048 g4096; do
  lib=$P/libmmseg_hip_$v.so; [ $v = g2048 ] && lib=$P/libmmseg_hip.so
  timeout -k 10 400 python3 $R/tools/benchlib.py $lib --model swin_unetr --size 128 --batch 1 --steps 20 --warmup 5 --no-cpu-baseline --timer-steps 2 > $O/c4_${v}_$i.log 2>&1 || { tail -20 $O/c4_${v}_$i.log; exit 1; }
  tail -1 $O/c4_${v}_$i.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); f=d['kernel_families']
print('== c4 $v', d['ms_per_step'], d['loss'], {k: f[k]['ms_per_step'] for k in f if 'head_dgrad' in k})"
  i=$((i+1))
done
bash $R/tools/gpu_check.sh r06zb || exit 1
echo r06zb done
