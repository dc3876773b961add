#!/bin/bash
# kernel durations + SQ counter passes of tools/stembench.py.  usage: bash tools/gpu_pmc_stem.sh TAG
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-ps}
mkdir -p $O
SB="python3 $R/tools/stembench.py --iters 10"
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t -o t -- $SB > $O/t.log 2>&1 || { tail -5 $O/t.log; exit 1; }
python3 $R/tools/kstats.py $O/t stem
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d $O/p1 -o pmc -- $SB > $O/p1.log 2>&1 || { tail -5 $O/p1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_INSTS_VMEM_WR --output-format csv -d $O/p2 -o pmc -- $SB > $O/p2.log 2>&1 || { tail -5 $O/p2.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/p3 -o pmc -- $SB > $O/p3.log 2>&1 || { tail -5 $O/p3.log; exit 1; }
python3 $R/tools/pmc_summary.py $O stem
