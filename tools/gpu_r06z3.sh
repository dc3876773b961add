#!/bin/bash
# r06z3: head data gradient with register-resident weights -- head tests, c4 trace (families) and bench line
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06z3
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest $R/tests/test_swin_unetr_gpu.py $R/tests/test_kernels_gpu.py -m gpu -x -q \
  -k "head or train_step" --timeout 240 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
[ $rc -ne 0 ] && { grep -E "^E " $O/tests.log | head -20; exit 1; }
B="python3 $R/bench.py --model swin_unetr --size 128 --batch 1"
timeout -k 10 600 rocprofv3 -M --kernel-trace --stats --output-format csv -d $O/trace -o prof -- $B --steps 10 --warmup 3 --timer-steps 1 --no-cpu-baseline > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 $R/tools/rocprof_families.py steady $O/trace/prof_kernel_trace.csv $O/steady.json 6 > $O/families.txt
grep -E "head|adamw" $O/families.txt
timeout -k 10 400 $B --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_c4.log 2>&1 || { tail -20 $O/bench_c4.log; exit 1; }
tail -1 $O/bench_c4.log | cut -c1-200
echo r06z3 done
