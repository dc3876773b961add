#!/bin/bash
# compile-time-M fusion forward (deferred encoder norm): parity tests, kernel durations, bench A/B vs the runtime-M kernel
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-fuse}
mkdir -p $O
[ -n "$SKIP_TESTS" ] || timeout -k 10 600 python3 -u -m pytest $R/tests -m gpu -x -q --timeout 300 --timeout-method thread -k "deferred or fuse or fusion or dual or bitwise or step_graph" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o prof -- python3 $R/bench.py --no-cpu-baseline --timer-steps 0 --steps 10 --warmup 3 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 $R/tools/kstats.py $O/prof fuse
bash $R/tools/gpu_ab.sh ${1:-fuse}_ab - MMSEG_FUSE_M=0 - MMSEG_FUSE_M=0
