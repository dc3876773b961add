#!/bin/bash
# r06r: window attention query pass with double-buffered LDS-DMA staging (A/B vs the previous build), swin GPU tests

set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06r
mkdir -p $O
cd $R
for v in old new old new; do
  if [ $v = old ]; then L="--lib $R/tools/_ab/lib_old.so"; else L=""; fi
  timeout -k 10 120 python3 tools/wabench.py --stages 0,1,2,3 $L > $O/wa_$v.log 2>&1 || { tail -20 $O/wa_$v.log; exit 1; }
  echo "== $v"; grep -E "stage|checksum" $O/wa_$v.log
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest $R/tests/test_swin_unetr_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $O/t.log 2>&1
rc=$?; tail -2 $O/t.log; grep -E "^E |FAILED" $O/t.log | head; echo "rc $rc"
