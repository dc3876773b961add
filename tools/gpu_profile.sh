#!/bin/bash
# One BASELINE config profiled end to end in one GPU call: a rocprofv3 kernel trace and three PMC passes (FETCH_SIZE,
# WRITE_SIZE, SQ; one counter group per run, no trace domains), each summary stamped with the run's workload key
# (bench.py --workload-out) so bench.py uses it only for that workload; then the judged bench line (with its CPU
# baseline), which reads those summaries.
#   usage: bash tools/gpu_profile.sh TAG CFG [bench args ...]      e.g.  r05a c4 --model swin_unetr --size 128 --batch 1
#   output: gpurun_out/TAG_CFG/{steady,pmc_traffic,pmc_sq}.json, bench.log, families_steady.txt, timer.json
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; CFG=$2; shift 2
O=$R/gpurun_out/${TAG}_${CFG}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py $* --workload-out $O/workload.json"
STEPS="--steps ${PROF_STEPS:-10} --warmup 3 --timer-steps 1 --no-cpu-baseline"
timeout -k 10 600 rocprofv3 -M --kernel-trace --stats --output-format csv -d $O/trace -o prof -- $B $STEPS > $O/prof.log 2>&1 || { echo "$CFG trace failed"; tail -20 $O/prof.log; exit 1; }
echo "$CFG trace ok"
PSTEPS="--steps 2 --warmup 1 --timer-steps 1 --no-cpu-baseline"
timeout -k 10 600 rocprofv3 -M --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o pmc -- $B $PSTEPS > $O/pmc_fetch.log 2>&1 || { echo "$CFG fetch failed"; tail -20 $O/pmc_fetch.log; exit 1; }
timeout -k 10 600 rocprofv3 -M --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o pmc -- $B $PSTEPS > $O/pmc_write.log 2>&1 || { echo "$CFG write failed"; tail -20 $O/pmc_write.log; exit 1; }
timeout -s KILL 300 rocprofv3 -M --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_sq -o pmc -- $B $PSTEPS > $O/pmc_sq.log 2>&1 || { echo "$CFG sq failed"; tail -20 $O/pmc_sq.log; exit 1; }
echo "$CFG pmc ok"
W="--workload $O/workload.json"
python3 $R/tools/rocprof_families.py steady $O/trace/prof_kernel_trace.csv $O/steady.json 6 $W > $O/families_steady.txt
python3 $R/tools/rocprof_families.py traffic $O/pmc_fetch/pmc_counter_collection.csv $O/pmc_write/pmc_counter_collection.csv $O/pmc_traffic.json $W > /dev/null
python3 $R/tools/rocprof_families.py sq $O/pmc_sq/pmc_counter_collection.csv $O/pmc_sq.json $W > /dev/null
# the judged line reads this call's summaries: stage them under profiles/ (collect_profile.sh keeps them locally)
cp $O/steady.json $R/profiles/${TAG}_${CFG}_steady.json && cp $O/pmc_traffic.json $R/profiles/${TAG}_${CFG}_pmc_traffic.json && cp $O/pmc_sq.json $R/profiles/${TAG}_${CFG}_pmc_sq.json
timeout -k 10 900 $B ${BENCH_STEPS:---steps 20 --warmup 5} --timer-dump $O/timer.json > $O/bench.log 2>&1 || { echo "$CFG bench failed"; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-400
echo "$CFG done"
