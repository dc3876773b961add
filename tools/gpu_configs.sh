#!/bin/bash
# bench lines of the BASELINE configs c2..c5 (1 GPU).  usage: bash tools/gpu_configs.sh TAG
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-cfg}
mkdir -p $O
run() { n=$1; shift; timeout -k 10 600 python3 $R/bench.py --no-cpu-baseline --timer-steps 1 "$@" > $O/$n.log 2>&1 || { tail -20 $O/$n.log; exit 1; }; tail -1 $O/$n.log | cut -c1-330; }
run c3 --steps 20 --warmup 5
run c2 --model unet --steps 20 --warmup 5
run c5 --modalities CT,PET,MRI --loss tversky --steps 20 --warmup 5
run c5fp8 --modalities CT,PET,MRI --loss tversky --fp8 --steps 20 --warmup 5
run c4 --model swin_unetr --size 128 --batch 1 --steps 5 --warmup 2
