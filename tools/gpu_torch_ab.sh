#!/bin/bash
# The same bench workload through the hardware.kernels: torch backend (PyTorch-ROCm ops, MIOpen convolutions):
# the reference's GPU mode (fp16 autocast + GradScaler) and bf16 autocast.  usage: bash tools/gpu_torch_ab.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-torch_ab}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for amp in fp16 bf16; do
  timeout -k 10 600 python3 -u $R/bench.py --kernels torch --amp $amp --steps 10 --warmup 3 > $O/bench_torch_$amp.log 2>&1 \
    || { echo "torch $amp bench failed"; tail -20 $O/bench_torch_$amp.log; exit 1; }
  tail -1 $O/bench_torch_$amp.log
done
