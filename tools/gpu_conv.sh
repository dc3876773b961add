#!/bin/bash
# conv microbench (+ optional SQ counter pass on one shape)
# usage: bash tools/gpu_conv.sh TAG [PMC]
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=${1:-c}
O=$R/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python3 $R/tools/convbench.py $CB_ARGS > $O/conv.log 2>&1 || { tail -20 $O/conv.log; exit 1; }
cat $O/conv.log
if [ -n "$2" ]; then
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $O/pmc1 -o pmc -- python3 $R/tools/convbench.py --shape $2 --iters 3 > $O/pmc1.log 2>&1 || { tail -20 $O/pmc1.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE --output-format csv -d $O/pmc2 -o pmc -- python3 $R/tools/convbench.py --shape $2 --iters 3 > $O/pmc2.log 2>&1 || { tail -20 $O/pmc2.log; exit 1; }
fi
echo done
