#!/bin/bash
# AdamW scalar tail folded into the vector launch: optimizer / step-graph / checkpoint tests + c3 bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04af
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest "$R/tests/test_kernels_gpu.py" "$R/tests/test_step_graph_gpu.py" "$R/tests/test_checkpoint_gpu.py" "$R/tests/test_dp_gpu.py" -k "adamw or graph or step or checkpoint or dp" -m gpu -q --timeout 600 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?
tail -2 $O/tests.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED" $O/tests.log | head -20; exit 1; }
timeout -k 10 600 python3 $R/bench.py --no-cpu-baseline > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['value'], [k for k in d['kernel_families'] if k.startswith('adamw')])"
