#!/bin/bash
# r04m: forced 24^3 grouping held to the pinned fp64 oracle, grouped tests, transposed-conv kernels; bench timer
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04m
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest "$R/tests/test_fullsize_gpu.py::test_fullsize_step_pinned_to_fp64_oracle" $R/tests/test_model_gpu.py::test_grouped_modalities_match_per_modality $R/tests/test_kernels_gpu.py::test_convT_fwd_dgrad_wgrad -m gpu -v -s --timeout 600 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
grep -E "pinned fp64|grouped from level" $O/tests.log | cut -c1-300
[ $rc -ne 0 ] && { grep -E "^E |FAILED" $O/tests.log | head -20; exit 1; }
timeout -k 10 600 python3 $R/bench.py --timer-dump $O/timer.json --no-cpu-baseline > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-160
