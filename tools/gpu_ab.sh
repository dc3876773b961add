#!/bin/bash
# Bench A/B over environment variants: bash tools/gpu_ab.sh TAG "VAR=1 VAR2=0" "VAR=0" ...  ("-" = defaults)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for v in "$@"; do
  e=$v; [ "$e" = "-" ] && e=""
  env $e timeout -k 10 300 python3 $R/bench.py --no-cpu-baseline --timer-steps 0 --steps ${AB_STEPS:-30} > $O/ab_$i.log 2>&1 || { tail -20 $O/ab_$i.log; exit 1; }
  echo "== [$v] $(tail -1 $O/ab_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
  i=$((i+1))
done
