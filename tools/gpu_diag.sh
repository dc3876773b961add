cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out/d1
cd $R
timeout -k 10 300 python3 tools/diag_tf.py unet_tiny 3 > gpurun_out/d1/brickr1.log 2>&1 || exit 1
MMSEG_BRICKR=0 timeout -k 10 300 python3 tools/diag_tf.py unet_tiny 3 > gpurun_out/d1/brickr0.log 2>&1 || exit 1
grep -c "<<<" gpurun_out/d1/brickr1.log gpurun_out/d1/brickr0.log
