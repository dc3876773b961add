#!/bin/bash
# InstanceNorm microbenchmark A/B over env variants (kernel trace per variant).  usage: bash tools/gpu_inab.sh TAG SIZE C "VAR=.." ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; S=$2; C=$3; shift 3
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for v in "$@"; do
  e=$v; [ "$e" = "-" ] && e=""
  for kv in $e; do export $kv; done
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/v$i -o k -- python3 $R/tools/inbench.py --size $S --c $C --iters 5 > $O/v$i.log 2>&1 || { tail -5 $O/v$i.log; exit 1; }
  for kv in $e; do unset ${kv%%=*}; done
  echo "== [$v]"
  python3 $R/tools/trace_runs.py $O/v$i/k_kernel_trace.csv | grep -v "at::native" | awk '{ if (!seen[$1" "$3]++) print }' | head -12
  i=$((i+1))
done
