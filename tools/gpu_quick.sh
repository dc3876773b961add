#!/bin/bash
# quick GPU iteration: all GPU tests (one process), then a short bench and optional kbench A/B.
# usage: bash tools/gpu_quick.sh TAG ["KNOB=a,b" ...]
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=${1:-q}; shift
O=$R/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python3 -m pytest $R/tests -m gpu -q -x > $O/tests.log 2>&1; rc=$?; tail -5 $O/tests.log
[ $rc -le 1 ] || exit 1
timeout -k 10 300 python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/bench.log 2>&1 || exit 1
tail -1 $O/bench.log
if [ -n "$PROF" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o prof -- python3 $R/bench.py --steps 10 --warmup 3 --timer-steps 0 --no-cpu-baseline > $O/prof.log 2>&1 || exit 1
  python3 $R/tools/rocprof_families.py stats $O/trace/prof_kernel_stats.csv 13 > $O/families.txt; head -32 $O/families.txt
fi
if [ $# -gt 0 ]; then
  timeout -k 10 600 python3 $R/tools/kbench.py --variants "$@" > $O/kbench.log 2>&1 || exit 1
  tail -30 $O/kbench.log
fi
