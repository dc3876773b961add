# r05h: DP rehearsal with SUM at world 1 (AVG is the identity there) vs AVG; bitwise DP test
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r05h; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest $R/tests/test_dp_gpu.py -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/tests.log | head -20; exit 1; }
run() { n=$1; shift; timeout -k 10 600 python3 $R/bench.py --no-cpu-baseline --timer-steps 1 --steps 40 "$@" > $O/$n.log 2>&1 || { tail -20 $O/$n.log; exit 1; }; python3 -c "
import json; d=json.loads(open('$O/$n.log').read().strip().splitlines()[-1]); print('$n', d['ms_per_step'], d['config']['parallelism'])"; }
for i in 1 2; do
  run plain$i
  run dp32sum_$i --dp-rehearsal --bucket-mb 32
  MMSEG_DP_AVG1=1 run dp32avg_$i --dp-rehearsal --bucket-mb 32
  run dp160sum_$i --dp-rehearsal --bucket-mb 160
done
timeout -k 10 600 rocprofv3 -M --kernel-trace --output-format csv -d $O/dptrace -o prof -- python3 $R/bench.py --no-cpu-baseline --dp-rehearsal --steps 10 --warmup 3 --timer-steps 1 > $O/dptrace.log 2>&1 || { tail -20 $O/dptrace.log; exit 1; }
python3 $R/tools/rocprof_families.py steady $O/dptrace/prof_kernel_trace.csv $O/dp_steady.json 6 > $O/dp_families.txt
grep -E "last|Reduce|reduce" $O/dp_families.txt
echo done
