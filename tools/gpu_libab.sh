#!/bin/bash
# A/B of two in-tree builds of libmmseg_hip (MMSEG_LIB_PATH) on convbench shapes, rocprofv3-timed.
# usage: bash tools/gpu_libab.sh TAG OPS shapes...   (builds: libmmseg_hip_ref.so = A, libmmseg_hip.so = B)
R=$GRAFT_REPO_ROOT
TAG=$1; OPS=$2; shift 2
P=$R/multimodal-organ-segmentation_amd
for v in ref new; do
  if [ $v = ref ]; then export MMSEG_LIB_PATH=$P/libmmseg_hip_ref.so; else export MMSEG_LIB_PATH=$P/libmmseg_hip.so; fi
  bash $R/tools/gpu_cbprof.sh ${TAG}_$v MMSEG_LIBAB "$v" $OPS "$@" || exit 1
done
