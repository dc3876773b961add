#!/bin/bash
# One GPU call: parity tests, the default bench, a rocprofv3 kernel-trace profile
# and three PMC passes (FETCH_SIZE, WRITE_SIZE, SQ MFMA-busy; separate runs, no trace domains).
# usage: bash tools/gpu_round.sh TAG [tests|notests]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r01}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
if [ "${2:-tests}" = "tests" ]; then
  timeout -k 10 900 python3 -u -m pytest $R/tests -m gpu -q -s --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
  rc=$?
  tail -3 $O/gpu_tests.log
  # 1 = some test assertions failed (keep measuring); anything else (abort, segfault, timeout) ends the call
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests ended with $rc"; tail -30 $O/gpu_tests.log; exit 1; fi
fi
timeout -k 10 600 python3 $R/bench.py --timer-dump $O/timer.json > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o prof -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/prof.log 2>&1 || { echo "prof failed"; tail -20 $O/prof.log; exit 1; }
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o pmc -- python3 $R/bench.py --steps 2 --warmup 1 --timer-steps 1 --no-cpu-baseline > $O/pmc_fetch.log 2>&1 || { echo "pmc fetch failed"; tail -20 $O/pmc_fetch.log; exit 1; }
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o pmc -- python3 $R/bench.py --steps 2 --warmup 1 --timer-steps 1 --no-cpu-baseline > $O/pmc_write.log 2>&1 || { echo "pmc write failed"; tail -20 $O/pmc_write.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_sq -o pmc -- python3 $R/bench.py --steps 2 --warmup 1 --timer-steps 1 --no-cpu-baseline > $O/pmc_sq.log 2>&1 || { echo "pmc sq failed"; tail -20 $O/pmc_sq.log; exit 1; }
python3 $R/tools/rocprof_families.py sq $O/pmc_sq/pmc_counter_collection.csv $O/pmc_sq.json > /dev/null
python3 $R/tools/rocprof_families.py stats $O/trace/prof_kernel_stats.csv 16 > $O/families.txt
python3 $R/tools/rocprof_families.py steady $O/trace/prof_kernel_trace.csv $O/steady.json 8 > $O/families_steady.txt
python3 $R/tools/rocprof_families.py traffic $O/pmc_fetch/pmc_counter_collection.csv $O/pmc_write/pmc_counter_collection.csv $O/pmc_traffic.json 4 > /dev/null
# the bench line again, now reading THIS call's trace / counter summaries (the names collect_round.sh gives them
# under profiles/), so its rocprof_* / traffic / mfma_busy fields come from the same tree and box
cp $O/steady.json $R/profiles/${TAG}_steady.json && cp $O/pmc_traffic.json $R/profiles/${TAG}_pmc_traffic.json && cp $O/pmc_sq.json $R/profiles/${TAG}_pmc_sq.json
timeout -k 10 600 python3 $R/bench.py > $O/bench_final.log 2>&1 || { echo "final bench failed"; tail -20 $O/bench_final.log; exit 1; }
tail -1 $O/bench_final.log
echo done
