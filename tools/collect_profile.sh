#!/bin/bash
# Keep the judged files of one tools/gpu_profile.sh call (run locally after gpurun):
#   profiles/TAG_CFG_{steady,pmc_traffic,pmc_sq}.json (staged by the call itself), TAG_CFG_bench.json (the judged
#   line), TAG_CFG_families_steady.txt, TAG_CFG_timer.txt.      usage: bash tools/collect_profile.sh TAG CFG...
set -e
T=$1; shift
for C in "$@"; do
  O=gpurun_out/${T}_$C
  P=profiles/${T}_$C
  for k in steady pmc_traffic pmc_sq; do [ -f $O/$k.json ] && cp $O/$k.json ${P}_$k.json; done
  [ -f $O/bench.log ] && tail -1 $O/bench.log > ${P}_bench.json
  [ -f $O/families_steady.txt ] && cp $O/families_steady.txt ${P}_families_steady.txt
  [ -f $O/timer.json ] && python3 tools/timer_dump.py $O/timer.json 40 > ${P}_timer.txt
  ls ${P}_*
done
