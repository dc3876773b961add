# r05z2: c3 A/B of the deferred-norm weight gradient on LDS-DMA staging (MMSEG_WGRAD_DMA_NORM=1) vs the pipelined register-staged kernel
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r05z2; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
for p in 0 1 0 1; do
  MMSEG_WGRAD_DMA_NORM=$p timeout -k 10 300 python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --timer-steps 1 --timer-dump $O/timer_$p.json > $O/bench_$p.log 2>&1 || { tail -20 $O/bench_$p.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/bench_$p.log').read().strip().splitlines()[-1]); print('dma_norm $p c3', d['ms_per_step'], d['value'], d['roofline']['kernel'], d['roofline']['avg_launch_ms'], d['roofline']['frac'])"
  python3 $R/tools/timer_families.py $O/timer_$p.json 60 | grep -E "wgrad_brick2|wgrad_dma|launches"
done
