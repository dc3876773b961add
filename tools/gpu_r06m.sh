#!/bin/bash
# r06m: chunk-major grouped IN backward grids: grouped-modality tests, c3 / c5 bench lines
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06m
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest $R/tests/test_model_gpu.py $R/tests/test_fullsize_gpu.py -m gpu -q -x -k "group or pinned or fullsize" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/t.log 2>&1
rc=$?; tail -2 $O/t.log; grep -E "^E |FAILED" $O/t.log | head; [ $rc -gt 1 ] && exit 1
cd $R
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/c3.log 2>&1 || { tail -20 $O/c3.log; exit 1; }
timeout -k 10 300 python3 bench.py --modalities CT,PET,MRI --loss tversky --steps 20 --warmup 5 --no-cpu-baseline > $O/c5.log 2>&1 || { tail -20 $O/c5.log; exit 1; }
for c in c3 c5; do python3 -c "
import json; d=json.loads(open('$O/$c.log').read().strip().split('\n')[-1]); f=d['kernel_families']
print('$c', d['ms_per_step'], d['value'], {k: f[k]['ms_per_step'] for k in ('in_bwd_partial','in_bwd_apply') if k in f})"; done
echo r06m done
