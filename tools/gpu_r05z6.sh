# r05z6: fp8 tests with the brick2 routing pinned; grouping-mode gradient differences per knob (tools/diag_force.py)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r05z6; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest $R/tests/test_fp8_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/tests.log | head -20; exit 1; }
cd $R && timeout -k 10 600 python3 -u tools/diag_force.py - MMSEG_WGRAD_B2_PIPE=0 MMSEG_WRED_V4=0 MMSEG_BRICK2_MINUNITS=0 MMSEG_WGRAD_PDIRECT=0 2>&1 | tee $O/diag.log | grep -v Warning
