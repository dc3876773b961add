#!/bin/bash
# r06o: rocprofv3 kernel trace of the window-attention microbench (per-kernel split of the c4 stage shapes)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06o
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o wa -- python3 $R/tools/wabench.py --stages 0,1,2,3 --reps 10 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
f=$(find $O/prof -name "wa_kernel_stats.csv" | head -1); cut -d, -f1-6 "$f" | head -20
python3 - "$O" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/prof/**/wa_kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
seq = [(r["Kernel_Name"][:60], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3) for r in rows if "winattn" in r["Kernel_Name"]]
agg = collections.defaultdict(list)
for i, (k, t) in enumerate(seq):
    agg[k].append(t)
for k, v in agg.items():
    print(f"{k:60s} n={len(v):4d} " + " ".join(f"{x:.1f}" for x in v[:14]))
PY
echo r06o done
