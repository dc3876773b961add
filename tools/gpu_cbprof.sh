#!/bin/bash
# A/B one env knob on convbench shapes with GPU-side kernel durations (rocprofv3 kernel trace; convbench's own
# HIP-event numbers are host-bound for launches under ~40 us).
# usage: bash tools/gpu_cbprof.sh TAG KNOB "vals" OPS shapes...
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=$1; KNOB=$2; VALS=$3; OPS=$4; shift 4
O=$R/gpurun_out/$TAG
mkdir -p $O
for v in $VALS; do
  for sh in "$@"; do
    export $KNOB=$v
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p_${v}_${sh} -o p -- python3 $R/tools/convbench.py --shape $sh --only $OPS --iters 20 > $O/log_${v}_${sh}.txt 2>&1 || { echo "fail $v $sh"; tail -5 $O/log_${v}_${sh}.txt; exit 1; }
    echo "== $KNOB=$v shape $sh"
    python3 - "$O/p_${v}_${sh}" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/p_kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    n = r["Name"]
    if "at::" in n or "rocclr" in n:
        continue
    print(f"   {n[:70]:70s} calls={r['Calls']:>4s} avg={float(r['AverageNs'])/1e3:8.2f} us")
PY
  done
done
