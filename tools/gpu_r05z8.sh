# r05z8: what bounds c3's deferred-norm 32-co brick weight gradient: full / no loads after the first brick (DBG=1) /
# no MFMA (DBG=2), pipelined and not (probe build, tools/convbench.py)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r05z8; mkdir -p $O; cd $R
for p in 1 0; do for d in 0 1 2; do
  MMSEG_WGRAD_B2_PIPE=$p MMSEG_WGRAD_DBG=$d timeout -k 10 120 python3 tools/convbench.py --lib libmmseg_hip_probe.so --shape 2,96,32,32 --only wgradn,wgrad --iters 30 2>&1 | grep "{" | sed "s/^/pipe $p dbg $d /" | tee -a $O/probe.log
done; done
