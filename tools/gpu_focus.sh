#!/bin/bash
# One GPU call for a subset of the GPU tests, then (unless "notbench") the default bench, a rocprofv3 kernel
# trace of the same bench and the SQ MFMA-busy PMC pass.
# usage: bash tools/gpu_focus.sh TAG "tests/test_a.py tests/test_b.py::name" [bench|nobench]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-focus}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
if [ -n "$2" ]; then
  T=""
  for t in $2; do T="$T $R/$t"; done
  timeout -k 10 1000 python3 -u -m pytest $T -m gpu -v -s --timeout 900 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
  rc=$?
  tail -3 $O/gpu_tests.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests ended with $rc"; tail -30 $O/gpu_tests.log; exit 1; fi
fi
if [ "${3:-bench}" = "bench" ]; then
  timeout -k 10 600 python3 $R/bench.py --timer-dump $O/timer.json > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
  tail -1 $O/bench.log
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o prof -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/prof.log 2>&1 || { echo "prof failed"; tail -20 $O/prof.log; exit 1; }
  tail -1 $O/prof.log
  timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_sq -o pmc -- python3 $R/bench.py --steps 2 --warmup 1 --timer-steps 1 --no-cpu-baseline > $O/pmc_sq.log 2>&1 || { echo "pmc sq failed"; tail -20 $O/pmc_sq.log; exit 1; }
  python3 $R/tools/rocprof_families.py sq $O/pmc_sq/pmc_counter_collection.csv $O/pmc_sq.json > /dev/null
  python3 $R/tools/rocprof_families.py stats $O/trace/prof_kernel_stats.csv 16 > $O/families.txt
  python3 $R/tools/rocprof_families.py steady $O/trace/prof_kernel_trace.csv $O/steady.json 8 > $O/families_steady.txt
fi
echo done
