# r05x (final, c4 again after the compile-time window tiles): per-config profile and judged bench line: c4
set -o pipefail
R=$GRAFT_REPO_ROOT
PROF_STEPS=6 BENCH_STEPS="--steps 5 --warmup 2 --cpu-steps 1" bash $R/tools/gpu_profile.sh r05x c4 --model swin_unetr --size 128 --batch 1 || exit 1
echo done
