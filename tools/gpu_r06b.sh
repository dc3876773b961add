#!/bin/bash
# r06b: the row-slab weight-gradient kernel: parity (kernel, deferred norm, full-size pinned steps), convbench A/B
# against the brick kernels, c3 bench A/B; the envelope Dice gates
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06b
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
PT="python3 -u -m pytest -q -s --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $PT $R/tests/test_kernels_gpu.py -k "wgrad_row" > $O/t_row.log 2>&1
rc=$?; tail -2 $O/t_row.log; grep -E "wgrad_row \(|^E |FAILED" $O/t_row.log | head -30
[ $rc -gt 1 ] && exit 1
[ $rc -eq 1 ] && exit 1
timeout -k 10 900 $PT $R/tests/test_model_gpu.py $R/tests/test_fullsize_gpu.py $R/tests/test_dice_heldout_gpu.py $R/tests/test_step_graph_gpu.py > $O/t_model.log 2>&1
rc=$?; tail -2 $O/t_model.log; grep -E "^E |FAILED|held-out|free-running|envelope" $O/t_model.log | head -30
[ $rc -gt 1 ] && exit 1
cd $R
for ROW in 1 0; do
  MMSEG_WGRAD_ROW=$ROW timeout -k 10 300 python3 tools/convbench.py --shape 2,96,32,32 2,96,64,32 --only wgrad,wgradn --iters 30 > $O/cb_row$ROW.log 2>&1 || { tail -5 $O/cb_row$ROW.log; exit 1; }
  echo "row=$ROW"; grep -v amdgpu.ids $O/cb_row$ROW.log | cut -c1-300
done
for ROW in 1 0 1; do
  MMSEG_WGRAD_ROW=$ROW timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_row$ROW.log 2>&1 || { tail -5 $O/bench_row$ROW.log; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('$O/bench_row$ROW.log').read().strip().split('\n')[-1])
f=d['kernel_families']; print('row=$ROW', d['ms_per_step'], 'graphs', d.get('captured_graphs'), d['roofline']['kernel'], d['roofline']['frac'], {k: v for k, v in f.items() if 'wgrad' in k})"
done
echo r06b done
