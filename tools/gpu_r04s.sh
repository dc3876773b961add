#!/bin/bash
# deferred weight-gradient reduces flushed once the queued partials pass N MB (MMSEG_WRED_FLUSH_MB): c3 A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
AB_STEPS=40 bash $R/tools/gpu_ab.sh r04s_ab - MMSEG_WRED_FLUSH_MB=60 MMSEG_WRED_FLUSH_MB=120 MMSEG_WRED_FLUSH_MB=240 - MMSEG_WRED_FLUSH_MB=60 MMSEG_WRED_FLUSH_MB=120 MMSEG_WRED_FLUSH_MB=240
