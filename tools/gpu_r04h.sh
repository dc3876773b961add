#!/bin/bash
# r04h: batched-reduce bitwise test + A/B; c4 with / without the window-summed score gradient
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04h
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest $R/tests/test_model_gpu.py::test_batched_weight_gradient_reduce_bitwise $R/tests/test_model_gpu.py::test_grouped_modalities_match_per_modality $R/tests/test_step_graph_gpu.py -m gpu -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
[ $rc -ne 0 ] && { grep -E "^E |Error" $O/tests.log | head -20; exit 1; }
AB_STEPS=40 bash $R/tools/gpu_ab_file.sh r04h_ab tools/ab_r04h.txt || exit 1
for v in 1 0; do
  MMSEG_WINATTN_SUM=$v timeout -k 10 600 python3 $R/bench.py --model swin_unetr --size 128 --batch 1 --steps 5 --warmup 2 --no-cpu-baseline --timer-steps 1 > $O/c4_sum$v.log 2>&1 || { tail -20 $O/c4_sum$v.log; exit 1; }
  echo "c4 MMSEG_WINATTN_SUM=$v $(tail -1 $O/c4_sum$v.log | cut -c1-200)"
done
