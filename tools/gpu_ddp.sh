#!/bin/bash
# DP rehearsal on one GPU: bench.py through torchrun with 2 ranks sharing cuda:0 over gloo, then 1 rank over
# RCCL (the driver's N>1 launch line), each under its own time limit.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ddp
mkdir -p $O
MMSEG_DIST_BACKEND=gloo timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 $R/bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline > $O/gloo2.log 2>&1 || { echo "gloo2 failed"; tail -30 $O/gloo2.log; exit 1; }
grep '"metric"' $O/gloo2.log | cut -c1-300
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29532 $R/bench.py --gpus 1 --steps 5 --warmup 2 --no-cpu-baseline > $O/rccl1.log 2>&1 || { echo "rccl1 failed"; tail -30 $O/rccl1.log; exit 1; }
grep '"metric"' $O/rccl1.log | cut -c1-300
