#!/bin/bash
# r06f: whole GPU suite after the second pruning pass (r04 window-attention kernels, wgrad ring, 30 switches), smoke, c3 bench line
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06f
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest $R/tests -m gpu -q -s --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
rc=$?
tail -2 $O/gpu_tests.log
grep -E "^E |FAILED|free-running|envelope" $O/gpu_tests.log | head -30
[ $rc -gt 1 ] && { echo "suite rc $rc"; exit 1; }
cd $R && timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_c3.log 2>&1 || { tail -20 $O/bench_c3.log; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench_c3.log').read().strip().split('\n')[-1])
print(d['ms_per_step'], d['value'], 'graphs', d['captured_graphs'], d['roofline']['kernel'], d['roofline']['frac'])"
echo r06f done
