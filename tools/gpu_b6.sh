#!/bin/bash
# brick6 vs brick5 on the 96^3 32->32 layers (convbench, variants interleaved) and the parity tests that cover
# the v5/v6 paths.  usage: bash tools/gpu_b6.sh TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-b6}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in "MMSEG_BRICK6=0" "MMSEG_BRICK6=1" "MMSEG_BRICK6=0" "MMSEG_BRICK6=1"; do
  env $v timeout -k 10 120 python3 -u $R/tools/convbench.py --iters 30 --only fwd,fwdn --shape 2,96,32,32 > $O/cb.log 2>&1 || { tail -20 $O/cb.log; exit 1; }
  echo "== $v"; grep -v amdgpu.ids $O/cb.log
done
timeout -k 10 120 python3 -u $R/tools/convbench.py --probe --iters 20 --only fwd,fwdn --shape 2,96,32,32 > $O/tl.log 2>&1 || { tail -20 $O/tl.log; exit 1; }
grep -v amdgpu.ids $O/tl.log
timeout -k 10 600 python3 -u -m pytest $R/tests/test_kernels_gpu.py $R/tests/test_model_gpu.py $R/tests/test_fullsize_gpu.py -q -x --timeout 300 --timeout-method thread -p no:cacheprovider -k "variants or deferred_conv_norm or step_bitwise or teacher_forced_steps_pinned or fullsize_training or full_size_forward" > $O/tests.log 2>&1
rc=$?
tail -5 $O/tests.log
exit $rc
