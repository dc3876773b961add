#!/bin/bash
# r06za: head data gradient with 16-B weight loads (v1, the in-tree build) and additionally a 2,048-block grid (v2,
# libmmseg_hip_v2.so: 32 voxels per lane instead of 8) against the previous build: head tests on v1, then the c4
# step per build, interleaved, with the per-family timer
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06za
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest $R/tests/test_swin_unetr_gpu.py $R/tests/test_kernels_gpu.py -m gpu -x -q \
  -k "head or train_step" --timeout 240 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
[ $rc -ne 0 ] && { grep -E "^E " $O/tests.log | head -20; exit 1; }
P=$R/multimodal-organ-segmentation_amd
i=0
for v in prev v1 v2 prev v1 v2; do
  lib=$P/libmmseg_hip.so; [ $v = prev ] && lib=$P/libmmseg_hip_prev.so; [ $v = v2 ] && lib=$P/libmmseg_hip_v2.so
  timeout -k 10 400 python3 $R/tools/benchlib.py $lib --model swin_unetr --size 128 --batch 1 --steps 20 --warmup 5 --no-cpu-baseline --timer-steps 2 > $O/c4_${v}_$i.log 2>&1 || { tail -20 $O/c4_${v}_$i.log; exit 1; }
  tail -1 $O/c4_${v}_$i.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); f=d['kernel_families']
print('== c4 $v', d['ms_per_step'], d['loss'], {k: f[k]['ms_per_step'] for k in f if 'head' in k})"
  i=$((i+1))
done
echo r06za done
