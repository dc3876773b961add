#!/bin/bash
# Round-3 GPU call: selected tests, the default bench (graph-replayed step), host submit time, a rocprofv3
# kernel-trace profile of the bench.  usage: bash tools/gpu_r03.sh TAG "pytest -k expression"
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r03}
K=${2:-}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
if [ -n "$K" ]; then
  timeout -k 10 900 python3 -u -m pytest $R/tests -m gpu -k "$K" -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
  rc=$?
  tail -3 $O/tests.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests ended with $rc"; exit 1; fi
fi
timeout -k 10 600 python3 $R/bench.py > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log
for gr in 0 1; do
  MMSEG_STEP_GRAPH=$gr timeout -k 10 300 python3 $R/tools/hosttime.py > $O/hosttime_g$gr.log 2>&1 || { echo "hosttime failed"; tail -20 $O/hosttime_g$gr.log; exit 1; }
  echo "step graph $gr:"; cat $O/hosttime_g$gr.log
done
MMSEG_STEP_GRAPH=0 timeout -k 10 600 python3 $R/bench.py --no-cpu-baseline > $O/bench_eager.log 2>&1 || { echo "bench eager failed"; tail -20 $O/bench_eager.log; exit 1; }
echo "eager:"; tail -1 $O/bench_eager.log | cut -c1-400
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o prof -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/prof.log 2>&1 || { echo "prof failed"; tail -20 $O/prof.log; exit 1; }
find $O -name "*kernel_stats.csv" | head -3
echo done
