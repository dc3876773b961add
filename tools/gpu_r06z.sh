#!/bin/bash
# r06z: fused AdamW + weight pack -- its tests and the step-graph tests, then c3 / c4 bench lines
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06z
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest $R/tests/test_adamw_pack_gpu.py $R/tests/test_step_graph_gpu.py -m gpu -x -v \
  --timeout 240 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?
tail -15 $O/tests.log
[ $rc -ne 0 ] && { grep -E "^E " $O/tests.log | head -20; exit 1; }
cd $R
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_c3.log 2>&1 || { tail -20 $O/bench_c3.log; exit 1; }
tail -1 $O/bench_c3.log | cut -c1-200
timeout -k 10 400 python3 bench.py --model swin_unetr --size 128 --batch 1 --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_c4.log 2>&1 || { tail -20 $O/bench_c4.log; exit 1; }
tail -1 $O/bench_c4.log | cut -c1-200
echo r06z done
