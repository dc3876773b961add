# r05g: DP rehearsal (RCCL world 1, captured step) against the plain step, interleaved; bucket sizes; DP trace
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r05g; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
run() { n=$1; shift; timeout -k 10 600 python3 $R/bench.py --no-cpu-baseline --timer-steps 1 --steps 40 "$@" > $O/$n.log 2>&1 || { tail -20 $O/$n.log; exit 1; }; python3 -c "
import json; d=json.loads(open('$O/$n.log').read().strip().splitlines()[-1]); print('$n', d['ms_per_step'], d['config']['parallelism'])"; }
for i in 1 2; do
  run plain$i
  run dp32_$i --dp-rehearsal --bucket-mb 32
  run dp64_$i --dp-rehearsal --bucket-mb 64
  run dp160_$i --dp-rehearsal --bucket-mb 160
done
MMSEG_DP_WRED_BATCH=0 run dp32_nobatch --dp-rehearsal --bucket-mb 32
timeout -k 10 600 rocprofv3 -M --kernel-trace --output-format csv -d $O/dptrace -o prof -- python3 $R/bench.py --no-cpu-baseline --dp-rehearsal --steps 10 --warmup 3 --timer-steps 1 > $O/dptrace.log 2>&1 || { tail -20 $O/dptrace.log; exit 1; }
python3 $R/tools/rocprof_families.py steady $O/dptrace/prof_kernel_trace.csv $O/dp_steady.json 6 > $O/dp_families.txt
head -14 $O/dp_families.txt
echo done
