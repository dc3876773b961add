#!/bin/bash
# SQ / LDS counter passes (one counter group per rocprofv3 run, no trace domains) on one convbench shape.
# usage: bash tools/gpu_pmc_conv.sh TAG SHAPE OP   (e.g. r02h 2,12,256,256 fwd); env knobs pass through
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-pc}
mkdir -p $O
CB="python3 $R/tools/convbench.py --shape $2 --only $3 --iters 5"
timeout -k 10 120 $CB > $O/conv.log 2>&1 || exit 1
tail -1 $O/conv.log
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d $O/p1 -o pmc -- $CB > $O/p1.log 2>&1 || { tail -5 $O/p1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM --output-format csv -d $O/p2 -o pmc -- $CB > $O/p2.log 2>&1 || { tail -5 $O/p2.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/p3 -o pmc -- $CB > $O/p3.log 2>&1 || { tail -5 $O/p3.log; exit 1; }
python3 $R/tools/pmc_summary.py $O conv3_ wgrad_
