#!/bin/bash
# r06z7: generic / token-linear weight gradient with two stages of loads in flight (wgrad_kernel, two register
# sets): pointbench and the c4 step against the previous build (libmmseg_hip_prev.so), interleaved; then the whole
# GPU suite on the new build.  Result: bitwise the same gradients, no faster (pointbench 594-599 vs 603-607 us,
# c4 17.43-17.44 vs 17.41-17.46 ms): not kept, the build reverted (profiles/r06z7_*)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06z7
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P=$R/multimodal-organ-segmentation_amd
i=0
for v in prev new prev new; do
  lib=$P/libmmseg_hip.so; [ $v = prev ] && lib=$P/libmmseg_hip_prev.so
  timeout -k 10 300 python3 $R/tools/pointbench.py --lib $lib --reps 20 > $O/point_${v}_$i.log 2>&1 || { tail -20 $O/point_${v}_$i.log; exit 1; }
  echo "== $v $(grep total $O/point_${v}_$i.log)"
  i=$((i+1))
done
for v in prev new prev new; do
  lib=$P/libmmseg_hip.so; [ $v = prev ] && lib=$P/libmmseg_hip_prev.so
  timeout -k 10 400 python3 $R/tools/benchlib.py $lib --model swin_unetr --size 128 --batch 1 --steps 20 --warmup 5 --no-cpu-baseline --timer-steps 0 > $O/c4_${v}_$i.log 2>&1 || { tail -20 $O/c4_${v}_$i.log; exit 1; }
  echo "== c4 $v $(tail -1 $O/c4_${v}_$i.log | cut -c1-130)"
  i=$((i+1))
done
bash $R/tools/gpu_check.sh r06z7 || exit 1
echo r06z7 done
