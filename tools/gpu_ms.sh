#!/bin/bash
# modality streams x split-K slot counts of the small-level kernels (kbench, eager steps, one process)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-ms}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 python3 -u $R/tools/kbench.py --variants "MMSEG_MODALITY_STREAMS=0,1" "MMSEG_BRICKR_SLOTS=256,128" "MMSEG_WGRAD_RSLOTS=256,128" --rounds 4 --steps 10 > $O/kb.log 2>&1 || { tail -20 $O/kb.log; exit 1; }
grep variant $O/kb.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l)
    print(d['variant'], d['median_ms'], d['min_ms'])"
