# r05x (final): whole GPU suite + smoke, then the c4 profile and judged line again (window-attention forward changed)
set -o pipefail
R=$GRAFT_REPO_ROOT
bash $R/tools/gpu_check.sh r05xchk4 || exit 1
PROF_STEPS=6 BENCH_STEPS="--steps 5 --warmup 2 --cpu-steps 1" bash $R/tools/gpu_profile.sh r05x c4 --model swin_unetr --size 128 --batch 1 || exit 1
echo done
