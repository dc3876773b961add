#!/bin/bash
# Kernel trace of the InstanceNorm microbenchmark at the 96^3 / 48^3 / 24^3 shapes.  usage: bash tools/gpu_inprof.sh TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-inprof}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for sc in "96 32" "48 64" "24 128" "12 256" "6 512"; do
  set -- $sc
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/s$1 -o k -- python3 $R/tools/inbench.py --size $1 --c $2 > $O/s$1.log 2>&1 || { tail -5 $O/s$1.log; exit 1; }
done
python3 $R/tools/trace_runs.py $O/s96/k_kernel_trace.csv $O/s48/k_kernel_trace.csv $O/s24/k_kernel_trace.csv $O/s12/k_kernel_trace.csv $O/s6/k_kernel_trace.csv
