#!/bin/bash
# A/B of one knob: conv tests (-k), convbench per value, and the bench per value.
# usage: bash tools/gpu_ab.sh TAG KNOB "v1 v2" [pytest -k expr] [convbench shapes]
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=$1; KNOB=$2; VALS=$3; KEXPR=${4:-conv3}; SHAPES=${5:-"2,96,32,32 2,96,64,32"}
O=$R/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest $R/tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$KEXPR" > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log
[ $rc -le 1 ] || exit 1
for v in $VALS; do
  env $KNOB=$v timeout -k 10 300 python3 $R/tools/convbench.py --shape $SHAPES --only fwd,dgrad > $O/conv_$v.log 2>&1 || { tail $O/conv_$v.log; exit 1; }
  echo "== $KNOB=$v"; cat $O/conv_$v.log
done
for v in $VALS; do
  env $KNOB=$v timeout -k 10 300 python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_$v.log 2>&1 || { tail $O/bench_$v.log; exit 1; }
  echo "== bench $KNOB=$v"; tail -1 $O/bench_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['value'], d['roofline']['kernel'], d['roofline']['frac'])"
done
