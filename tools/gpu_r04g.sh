#!/bin/bash
# r04g: kernel tests for the halo ring + summed window-attention score gradient, then the A/B list
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04g
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest $R/tests/test_kernels_gpu.py::test_wgrad_dma_halo_ring $R/tests/test_swin_unetr_gpu.py::test_window_attention_summed_score_gradient $R/tests/test_swin_unetr_gpu.py::test_fused_window_attention_vs_torch -m gpu -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?
tail -5 $O/tests.log
grep -E "window-summed" $O/tests.log
[ $rc -ne 0 ] && { grep -E "^E |Error" $O/tests.log | head -20; exit 1; }
AB_STEPS=40 bash $R/tools/gpu_ab_file.sh r04g_ab tools/ab_r04f.txt
