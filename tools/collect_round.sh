#!/bin/bash
# Copy the judged summaries of one gpu_round.sh call from gpurun_out/TAG into profiles/TAG_* (run locally).
# usage: bash tools/collect_round.sh TAG
set -e
T=$1
O=gpurun_out/$T
P=profiles
[ -f $O/bench.log ] && tail -1 $O/bench.log > $P/${T}_bench.json
# (gpu_round.sh's last bench run reads the call's own trace / counter summaries: the judged line)
[ -f $O/bench_final.log ] && tail -1 $O/bench_final.log > $P/${T}_bench.json
[ -f $O/families.txt ] && cp $O/families.txt $P/${T}_families.txt
[ -f $O/trace/prof_kernel_stats.csv ] && cp $O/trace/prof_kernel_stats.csv $P/${T}_kernel_stats.csv
[ -f $O/steady.json ] && cp $O/steady.json $P/${T}_steady.json && cp $O/families_steady.txt $P/${T}_families_steady.txt
[ -f $O/pmc_traffic.json ] && cp $O/pmc_traffic.json $P/${T}_pmc_traffic.json
[ -f $O/pmc_sq.json ] && cp $O/pmc_sq.json $P/${T}_pmc_sq.json
[ -f $O/timer.json ] && python3 tools/timer_dump.py $O/timer.json 40 > $P/${T}_timer.txt
[ -f $O/gpu_tests.log ] && grep -E "passed|failed|PASSED|FAILED|pinned fp64|held-out|free-running|c5 96|fp8 vs|grouped|Error" $O/gpu_tests.log | cut -c1-400 > $P/${T}_gpu_tests.txt || true
C=gpurun_out/${T}_cfg
if [ -d $C ]; then for f in $C/c*.log; do n=$(basename $f .log); tail -1 $f > $P/${T}_config_$n.json; done; fi
ls -la $P/${T}_*
