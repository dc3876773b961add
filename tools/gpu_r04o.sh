#!/bin/bash
# compile-time 4x8x8 / 4x4x8 runtime-brick instantiations: kernel + grouped parity, then A/B against the runtime-brick
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04o
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest "$R/tests/test_kernels_gpu.py::test_b32_halo_staging" "$R/tests/test_model_gpu.py" -k "b32_halo or group" -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED" $O/tests.log | head -20; exit 1; }
timeout -k 10 600 python3 -u -m pytest "$R/tests/test_fullsize_gpu.py::test_fullsize_step_pinned_to_fp64_oracle" -k "dual_c3-bfloat16-1 or dual_m3_c5-bfloat16-1" -m gpu -v -s --timeout 600 --timeout-method thread -p no:cacheprovider > $O/pinned.log 2>&1
rc=$?
tail -3 $O/pinned.log
grep -E "pinned fp64" $O/pinned.log | cut -c1-300
[ $rc -ne 0 ] && { grep -E "^E |FAILED" $O/pinned.log | head -20; exit 1; }
AB_STEPS=40 bash $R/tools/gpu_ab.sh r04o_ab - MMSEG_BRICKR_CT488=0 - MMSEG_BRICKR_CT488=0
