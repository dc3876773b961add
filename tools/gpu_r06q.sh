#!/bin/bash
# r06q: SQ counters of the window-attention kernels at c4's stage-0 shape (one counter group per rocprofv3 run)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06q
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE --output-format csv -d $O/p1 -o pmc -- python3 $R/tools/wabench.py --stages 0 --reps 3 > $O/p1.log 2>&1 || { tail -20 $O/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE --output-format csv -d $O/p2 -o pmc -- python3 $R/tools/wabench.py --stages 0 --reps 3 > $O/p2.log 2>&1 || { tail -20 $O/p2.log; exit 1; }
python3 - "$O" <<'PY'
import csv, glob, sys, collections
for p in ("p1", "p2"):
    f = glob.glob(sys.argv[1] + f"/{p}/**/pmc_counter_collection.csv", recursive=True)[0]
    agg = collections.defaultdict(lambda: collections.defaultdict(float)); cnt = collections.Counter()
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "winattn" not in k: continue
        k = k.split("::")[-1][:28]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[(k, r["Counter_Name"])] += 1
    for k, d in agg.items():
        print(p, k, {c: round(v / max(1, cnt[(k, c)]) , 1) for c, v in d.items()})
PY
echo r06q done
