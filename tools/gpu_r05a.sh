set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r05a; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest $R/tests/test_step_graph_gpu.py $R/tests/test_dp_gpu.py "$R/tests/test_fullsize_gpu.py::test_group_force_runs_other_kernels" -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -le 1 ] || exit 1
timeout -k 10 600 python3 $R/bench.py --no-cpu-baseline > $O/c3.log 2>&1 || { tail -20 $O/c3.log; exit 1; }
tail -1 $O/c3.log | cut -c1-300
timeout -k 10 600 python3 $R/bench.py --no-cpu-baseline --dp-rehearsal > $O/c3dp.log 2>&1 || { tail -20 $O/c3dp.log; exit 1; }
tail -1 $O/c3dp.log | cut -c1-300
timeout -k 10 600 python3 $R/bench.py --no-cpu-baseline > $O/c3b.log 2>&1 || { tail -20 $O/c3b.log; exit 1; }
tail -1 $O/c3b.log | cut -c1-300
BENCH_STEPS="--steps 5 --warmup 2 --cpu-steps 1" bash $R/tools/gpu_profile.sh r05a c4 --model swin_unetr --size 128 --batch 1
