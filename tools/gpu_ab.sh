#!/bin/bash
# Bench A/B over variants: bash tools/gpu_ab.sh TAG "VAR=1 VAR2=0" "VAR=0 --fresh-inputs" ...  ("-" = defaults;
# tokens starting with -- are bench.py arguments, the rest environment assignments)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for v in "$@"; do
  envs=""; args=""
  if [ "$v" != "-" ]; then
    for tok in $v; do case $tok in --*) args="$args $tok";; *) envs="$envs $tok";; esac; done
  fi
  env $envs timeout -k 10 300 python3 $R/bench.py --no-cpu-baseline --timer-steps 0 --steps ${AB_STEPS:-30} $args > $O/ab_$i.log 2>&1 || { tail -20 $O/ab_$i.log; exit 1; }
  echo "== [$v] $(tail -1 $O/ab_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
  i=$((i+1))
done
