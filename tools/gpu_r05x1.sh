# r05x (final): per-config rocprofv3 trace + PMC summaries (workload-stamped) and judged bench lines: c3, c2
set -o pipefail
R=$GRAFT_REPO_ROOT
bash $R/tools/gpu_profile.sh r05x c3 || exit 1
bash $R/tools/gpu_profile.sh r05x c2 --model unet || exit 1
echo done
