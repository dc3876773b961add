#!/bin/bash
# mixed bf16/fp8 (config c5): parity tests, the brick6 tests, c5 bench in bf16 and bf16+fp8
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-fp8}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest $R/tests/test_fp8_gpu.py $R/tests/test_kernels_gpu.py $R/tests/test_model_gpu.py -q -x -s --timeout 300 --timeout-method thread -p no:cacheprovider -k "fp8 or variants or deferred_conv_norm or step_bitwise" > $O/tests.log 2>&1
rc=$?
tail -2 $O/tests.log; grep "fp8 vs bf16" $O/tests.log
[ $rc -ne 0 ] && { grep -E "^E |Error" $O/tests.log | head -8; exit $rc; }
for f in "" "--fp8" "" "--fp8"; do
  timeout -k 10 300 python3 $R/bench.py --modalities CT,PET,MRI --loss tversky --no-cpu-baseline --timer-steps 2 --steps 20 $f > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
  tail -1 $O/bench.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
print('$f', d['dtype'], d['ms_per_step'], d['value'], d['loss'], {k: v['ms_per_step'] for k, v in d['kernel_families'].items() if 'brick6' in k or 'F8' in k})"
done
