#!/bin/bash
# r06s: timing-only experiment -- a window-attention pass with staging only (2) / compute only (3), rocprofv3 per-kernel times
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06s
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in 0 2 3; do
  MMSEG_WA_EXP=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p$v -o wa -- python3 $R/tools/wabench.py --stages 0 --reps 5 > $O/p$v.log 2>&1 || { tail -5 $O/p$v.log; exit 1; }
  f=$(find $O/p$v -name "wa_kernel_stats.csv" | head -1); echo "== $v"; grep winattn "$f" | cut -d, -f1-4 | cut -c1-140
done
