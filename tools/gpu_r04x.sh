#!/bin/bash
# fused head + loss: data gradient from bf16 hi + lo MFMAs as well (MMSEG_HEAD_BF16): tests, head microbench, c3 A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04x
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest "$R/tests/test_model_gpu.py" "$R/tests/test_kernels_gpu.py" -k "head" -m gpu -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
grep -E "worst gradient rel" $O/tests.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED" $O/tests.log | head -20; exit 1; }
timeout -k 10 600 python3 -u -m pytest "$R/tests/test_fullsize_gpu.py::test_fullsize_step_pinned_to_fp64_oracle" -k "dual_c3-bfloat16-1 or dual_m3_c5-bfloat16-1" -m gpu -v -s --timeout 600 --timeout-method thread -p no:cacheprovider > $O/pinned.log 2>&1
rc=$?
tail -2 $O/pinned.log
grep -E "pinned fp64" $O/pinned.log | cut -c1-300
[ $rc -ne 0 ] && { grep -E "^E |FAILED" $O/pinned.log | head -20; exit 1; }
for v in 0 1; do MMSEG_HEAD_BF16=$v timeout -k 10 120 python3 $R/tools/headbench.py --step-only > $O/hb_$v.log 2>&1 || { tail -20 $O/hb_$v.log; exit 1; }; echo "== HEAD_BF16=$v"; tail -4 $O/hb_$v.log; done
AB_STEPS=40 bash $R/tools/gpu_ab.sh r04x_ab - MMSEG_HEAD_BF16=0  - MMSEG_HEAD_BF16=0 
