#!/bin/bash
# r06z5: token-linear weight gradient A/B (wgrad_kernel<point> staging 64 vs 128 voxels per stage: two builds,
# interleaved; the kv128 library was a one-off build of conv_gemm.hip with the launch at KV = 128, not kept:
# profiles/r06z5_pointbench_*.log), then the c2 / c5 profile sets of the fused AdamW + pack tree
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06z5
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in base kv128 base kv128; do
  lib=$R/multimodal-organ-segmentation_amd/libmmseg_hip.so
  [ $v = kv128 ] && lib=$R/multimodal-organ-segmentation_amd/libmmseg_hip_kv128.so
  timeout -k 10 300 python3 $R/tools/pointbench.py --lib $lib --reps 20 > $O/point_$v.log 2>&1 || { tail -20 $O/point_$v.log; exit 1; }
  echo "== $v"; grep -E "wgrad|total" $O/point_$v.log | sed -E 's/ y .*//' 
done
bash $R/tools/gpu_profile.sh r06z5 c2 --model unet || exit 1
bash $R/tools/gpu_profile.sh r06z5 c5 --modalities CT,PET,MRI --loss tversky || exit 1
echo r06z5 done
