#!/bin/bash
# Bench A/B over the environment variants listed in a file, one per line ("-" = defaults, "#" comments), twice
# interleaved: bash tools/gpu_ab_file.sh TAG FILE
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1
mapfile -t V < <(grep -v '^#' $R/$2 | grep -v '^$')
bash $R/tools/gpu_ab.sh $TAG "${V[@]}" "${V[@]}"
